# Round 2 (re-entry) first GPU call: the whole -m gpu suite on the rebuilt tree,
# then the CRC-bank and parts ablations (8 GiB) that size the GCM levers.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r2b_pytest.log 2>&1
rc=$?; tail -3 gpurun_out/r2b_pytest.log; [ $rc -eq 0 ] || exit 1
bash scripts/gpu_ab_crcbank.sh && bash scripts/gpu_ab_parts.sh
