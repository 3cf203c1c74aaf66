# The whole GPU test suite + smoke, as the driver runs them at round end.
# usage: bash scripts/gpu_full_tests.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/full_$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 1000 python3 -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error' $out/pytest.log | head -20; exit 1; }
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 && tail -1 $out/smoke.log
