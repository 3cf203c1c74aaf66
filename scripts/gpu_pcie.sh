set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== default"; timeout -k 10 60 ./tools/pcie_duplex 512 8 || exit 1
echo "== HSA_ENABLE_SDMA=0"; HSA_ENABLE_SDMA=0 timeout -k 10 60 ./tools/pcie_duplex 512 8 || exit 1
echo "== chunks 64"; timeout -k 10 60 ./tools/pcie_duplex 512 64 || exit 1
echo "== HIP_FORCE_DEV_KERNARG etc none; GPU_MAX_HW_QUEUES=$GPU_MAX_HW_QUEUES"
