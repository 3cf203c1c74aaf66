# Round-4 call 44: the final tree as the round-end driver runs it (pytest -m
# gpu, smoke(), bench.py with no flags), plus the configs[1] rocprof stats.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4z || exit 1
out=gpurun_out/r4z; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $out/bench_seal_gcm.json 2> $out/bench_seal_gcm.err || { echo "bench failed"; tail -5 $out/bench_seal_gcm.err; exit 1; }
echo "bench: $(tail -1 $out/bench_seal_gcm.json | cut -c1-120)"
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_gcm -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 --steps 10 --warmup 2 > $out/prof_gcm.log 2>&1 && echo "prof ok"
