set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/prof_r1
export TMPDIR=/tmp
timeout -k 10 400 python bench.py > gpurun_out/r1_bench_full.log 2>&1
echo "bench rc=$?"; tail -3 gpurun_out/r1_bench_full.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_r1 -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --verify 0 > gpurun_out/r1_prof_bench.log 2>&1
echo "prof rc=$?"
find gpurun_out/prof_r1 -name "*stats*" | head
