# Round-end evidence on the final tree: all GPU tests, smoke, default bench, GCM open,
# rocprof stats of the default bench.  usage: bash scripts/gpu_final.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
tag=${1:-final}
out=gpurun_out/$tag
bash scripts/gpu_verify.sh $tag || exit 1
export TMPDIR=/tmp
timeout -k 10 420 python3 bench.py --mode open --no-cpu > $out/open_gcm.json 2> $out/open_gcm.err || { echo "open bench failed"; tail -5 $out/open_gcm.err; exit 1; }
tail -1 $out/open_gcm.json | cut -c1-200
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_gcm -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --verify 0 > $out/prof_gcm.log 2>&1 || { echo "prof failed"; tail -5 $out/prof_gcm.log; exit 1; }
grep gcm_main $out/prof_gcm/run_kernel_stats.csv | cut -c1-220
