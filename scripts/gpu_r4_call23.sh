# Round-4 call 23: the aggregator with two dispatchers per device
# (JFSX_AGG_PAIR=1, sibling contexts) against one, 20 and 32 threads sealing
# 4 MiB pinned host blocks; the GPU aggregator tests with the pair first.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4w; mkdir -p $out
export TMPDIR=/tmp
JFSX_AGG_PAIR=1 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_agg.py tests/test_shim_sequence.py -q --timeout 120 --timeout-method thread > $out/t_pair.log 2>&1
rc=$?; echo "pair tests rc $rc: $(tail -1 $out/t_pair.log)"; [ $rc -ne 0 ] && exit 1
run() { local name=$1; shift; timeout -k 10 400 python3 bench.py --mode agg --no-cpu "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -3 $out/$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'], d['config'].get('batches'), d['config'].get('mean_batch'))" $out/$name.json $name; }
run t20 --threads 20 && JFSX_AGG_PAIR=1 run t20p --threads 20 && run t32 --threads 32 && JFSX_AGG_PAIR=1 run t32p --threads 32 && JFSX_AGG_PAIR=1 run t20p2 --threads 20
