# LZ4 stage: bench lines for compress / decompress on text and
# random 4 MiB blocks (4 GiB batches) + rocprof kernel stats.
# usage: bash scripts/gpu_lz4.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/lz4_$1
mkdir -p $out
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 300 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-200)"; python3 -c "import json; d=json.loads(open('$out/bench_$name.json').read().strip().splitlines()[-1]); print('  kernel_ms', d['roofline']['kernel_avg_ms'], 'ratio', d['config']['ratio'], 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'])"; }
run lz4_text --mode lz4 --lz4-data text --steps 2 --warmup 1 && \
run lz4_random --mode lz4 --lz4-data random --steps 2 --warmup 1 && \
run unlz4_text --mode unlz4 --lz4-data text --steps 2 --warmup 1 && \
run unlz4_random --mode unlz4 --lz4-data random --steps 2 --warmup 1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --mode lz4 --lz4-data text --steps 2 --warmup 1 --no-cpu --verify 0 > $out/prof.log 2>&1 && echo prof ok
