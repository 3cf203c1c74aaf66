# Round-4 call 25: the host ring's smallest slot (JFSX_RING_MIN_MB, default 16)
# for the aggregator's tens-of-MiB batches, 20 and 32 threads; the bulk
# host-ingest line with the default and the 4 MiB setting.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4y; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 400 python3 bench.py --no-cpu "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -3 $out/$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/$name.json $name; }
run t20_16 --mode agg --threads 20 && JFSX_RING_MIN_MB=8 run t20_8 --mode agg --threads 20 && JFSX_RING_MIN_MB=4 run t20_4 --mode agg --threads 20 && \
run t32_16 --mode agg --threads 32 && JFSX_RING_MIN_MB=8 run t32_8 --mode agg --threads 32 && JFSX_RING_MIN_MB=4 run t32_4 --mode agg --threads 32 && \
run ingest_16 --mem host --steps 4 --warmup 1 && JFSX_RING_MIN_MB=4 run ingest_4 --mem host --steps 4 --warmup 1
