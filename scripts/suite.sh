# One parametrised GPU suite (replaces the per-call gpu_r4_call*.sh scripts).
# Every committed line under profiles/r5 names the suite step that made it.
#
# usage (on the GPU box, from the repo root; chain steps with &&):
#   bash scripts/suite.sh <tag> tests                        pytest -m gpu (one process)
#   bash scripts/suite.sh <tag> line <name> [bench args]     one bench.py JSON line -> bench_<name>.json
#   bash scripts/suite.sh <tag> prof <name> [bench args]     rocprofv3 --kernel-trace --stats of that line
#   bash scripts/suite.sh <tag> pmc <name> "<ctrs>" [args]   one rocprofv3 --pmc pass (--steps 1 --warmup 0)
#   bash scripts/suite.sh <tag> smoke                        __graft_entry__.smoke()
# Outputs land in gpurun_out/suite_<tag>/.  Each GPU step runs under its own
# time limit; a failing step returns non-zero so the && chain stops there.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
tag=$1
step=$2
shift 2
out=gpurun_out/suite_$tag
mkdir -p "$out"
export TMPDIR=/tmp
TL=${SUITE_TIMEOUT:-500}
case $step in
tests)
    timeout -k 10 ${TL} python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" \
        > "$out/pytest.log" 2>&1
    rc=$?
    tail -3 "$out/pytest.log"
    exit $rc ;;
smoke)
    timeout -k 10 ${TL} python3 -c 'import __graft_entry__ as g; g.smoke(); print("smoke ok")' > "$out/smoke.log" 2>&1
    rc=$?
    tail -2 "$out/smoke.log"
    exit $rc ;;
line)
    name=$1; shift
    echo "bench.py $*" > "$out/bench_$name.cmd"
    timeout -k 10 ${TL} python3 -u bench.py "$@" > "$out/bench_$name.json" 2> "$out/bench_$name.err"
    rc=$?
    if [ $rc -ne 0 ]; then echo "$name failed ($rc)"; tail -5 "$out/bench_$name.err"; exit $rc; fi
    echo "$name: $(tail -1 "$out/bench_$name.json" | cut -c1-200)" ;;
prof)
    name=$1; shift
    echo "rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --verify 0 $*" > "$out/prof_$name.cmd"
    timeout -k 10 ${TL} rocprofv3 --kernel-trace --stats -d "$out/prof_$name" -o run --output-format csv \
        -- python3 bench.py --no-cpu --verify 0 "$@" > "$out/prof_$name.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "prof $name failed ($rc)"; tail -5 "$out/prof_$name.log"; exit $rc; fi
    echo "prof $name ok" ;;
pmc)
    name=$1; ctr=$2; shift 2
    echo "rocprofv3 --kernel-trace --pmc $ctr -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 $*" \
        > "$out/pmc_$name.cmd"
    timeout -s KILL ${PMC_TIMEOUT:-240} rocprofv3 --kernel-trace --pmc $ctr -d "$out/pmc_$name" -o run \
        --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" \
        > "$out/pmc_$name.log" 2>&1
    rc=$?
    if [ $rc -ne 0 ]; then echo "pmc $name failed ($rc)"; grep -v "^ *@" "$out/pmc_$name.log" | tail -3; exit $rc; fi
    echo "pmc $name ok" ;;
*)
    echo "suite.sh: unknown step $step"; exit 2 ;;
esac
