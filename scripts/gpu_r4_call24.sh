# Round-4 call 24: the aggregator's batching window (bench --agg-window-us)
# at 20 and 32 threads sealing 4 MiB pinned host blocks.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4x; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 400 python3 bench.py --mode agg --no-cpu "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -3 $out/$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); c=d['config']; print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'], {k: c[k] for k in c if 'batch' in k or 'window' in k})" $out/$name.json $name; }
for w in 500 100 250 1000 2000; do run t20_w$w --threads 20 --agg-window-us $w || exit 1; done
for w in 500 100 1000; do run t32_w$w --threads 32 --agg-window-us $w || exit 1; done
