# Round-end style check of the current tree: every GPU test, smoke(), default bench.
# usage: bash scripts/gpu_verify.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
tag=${1:-verify}
out=gpurun_out/$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"; tail -4 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -5 $out/smoke.log; exit 1; }
echo "smoke: $(tail -1 $out/smoke.log)"
timeout -k 10 420 python bench.py > $out/bench.json 2> $out/bench.err || { echo "bench failed"; tail -5 $out/bench.err; exit 1; }
tail -1 $out/bench.json
