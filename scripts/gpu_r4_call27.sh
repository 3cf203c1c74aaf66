# Round-4 call 27: what the round-end driver runs, on the current tree --
# pytest -m gpu, smoke(), and bench.py with no flags (configs[1]) -- plus the
# rocprofv3 kernel stats of that same default command.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4f2 || exit 1
out=gpurun_out/r4f2; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail -5 $out/bench_default.err; exit 1; }
echo "bench: $(tail -1 $out/bench_default.json | cut -c1-200)"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $out/prof_default -o run --output-format csv -- python3 bench.py --no-cpu > $out/prof_default.log 2>&1 && echo "prof ok"
