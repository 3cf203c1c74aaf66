# CRC-verify kernel: byte-table slice-by-4 variant (JFSX_CRC_BYTE=1) against the
# nibble-table default -- parity of the variant on the CRC tests, then the
# same-box A/B at 64 GiB.  usage: bash scripts/gpu_r3_crcbyte.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ab_$1
mkdir -p $out
JFSX_LIB=juicefs_amd/_build/libjfsx_CRCBYTE.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -x -q -m gpu --timeout 120 --timeout-method thread > $out/crcbyte.pytest.log 2>&1 || { echo "crcbyte parity FAILED"; tail -15 $out/crcbyte.pytest.log; exit 1; }
echo "crcbyte parity: $(tail -1 $out/crcbyte.pytest.log)"
AB_REPS="1 2" bash scripts/gpu_ab.sh $1 "--mode crc" default=default crcbyte=CRCBYTE
