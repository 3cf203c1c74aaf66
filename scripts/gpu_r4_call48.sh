# Round-4 call 48: the per-object aggregator lines (20 / 32 threads sealing
# 4 MiB pinned host blocks) on the final build, with same-run CPU baselines.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_r4l2; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-120)"; }
run agg_gcm_t20 --mode agg --threads 20 && run agg_gcm_t32 --mode agg --threads 32
