# GPU parity suite + smoke, then (optional) a measurement section of the r3 suite.
# usage: bash scripts/gpu_r3_tests.sh <tag> [suite-section]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest.log; exit 1; }
echo "gpu tests: $(tail -1 $out/pytest.log)"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
echo "smoke: $(tail -1 $out/smoke.log)"
if [ $# -ge 2 ]; then bash scripts/gpu_r3_suite.sh $1 $2; fi
