set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
echo "== default"; timeout -k 10 90 ./tools/pcie_duplex 512 8 || exit 1
echo "== HSA_ENABLE_SDMA=0"; HSA_ENABLE_SDMA=0 timeout -k 10 90 ./tools/pcie_duplex 512 8 || exit 1
