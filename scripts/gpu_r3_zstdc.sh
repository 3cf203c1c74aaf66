# Round 3: the zstd level-1 encoder on the GPU (parity with the system
# libzstd), the compressor contract port, error diagnostics, and a first
# compress bench.  usage: bash scripts/gpu_r3_zstdc.sh <tag> [bench args]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
shift
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_zstdc.py tests/test_compress_contract.py tests/test_gpu_errors.py tests/test_gpu_zstd.py tests/test_abi.py > $out/pytest.log 2>&1
rc=$?
tail -5 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $out/pytest.log | head -30; exit 1; }
if [ $# -gt 0 ]; then
  timeout -k 10 600 python3 bench.py "$@" > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
  tail -1 $out/bench.json | cut -c1-400
fi
