# Round-4 call 34: the zstd GPU tests with the 5000-object round trip.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ac; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zstdc.py tests/test_gpu_zstd.py -q --timeout 120 --timeout-method thread > $out/t.log 2>&1
rc=$?; echo "rc $rc: $(tail -1 $out/t.log)"; grep -E "FAILED|Error" $out/t.log | head -5; exit $rc
