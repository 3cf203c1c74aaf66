# Phase split of the block-parallel zstd decoder (stamp build), kernel stats
# of the default build, then the GPU suite + smoke.  usage: bash scripts/gpu_r3_zst.sh <tag> [suite-section]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
JFSX_LIB=juicefs_amd/_build/libjfsx_ZSTAMP.so timeout -k 10 200 python3 scripts/zstd_stamps.py 512 > $out/stamps_par.txt 2>&1 || { echo "stamps failed"; tail -20 $out/stamps_par.txt; exit 1; }
cat $out/stamps_par.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_unzstd -o run --output-format csv -- python3 bench.py --mode unzstd --blocks 4096 --no-cpu --verify 0 --steps 3 --warmup 1 > $out/prof_unzstd.log 2>&1 || { echo "prof failed"; tail -5 $out/prof_unzstd.log; exit 1; }
echo "prof ok"
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest.log; exit 1; }
echo "gpu tests: $(tail -1 $out/pytest.log)"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
echo "smoke: $(tail -1 $out/smoke.log)"
if [ $# -ge 2 ]; then bash scripts/gpu_r3_suite.sh $1 $2; fi
