# Round 2, first GPU pass: the whole -m gpu suite, then the default bench line.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r2a
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -25 $out/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $out/bench.json 2> $out/bench.err
rc=$?
echo "bench rc=$rc"; tail -3 $out/bench.json; tail -5 $out/bench.err
exit $rc
