# Compression stage suite: 64 GiB bench lines with CPU
# baselines for LZ4 compress/decompress and zstd decompress (text / random),
# then rocprof kernel stats of the text lines.  usage: bash scripts/gpu_codec_suite.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/codec_$1
mkdir -p $out
export TMPDIR=/tmp
for m in ${MODES:-lz4 unlz4 unzstd}; do for d in text random; do
  timeout -k 10 500 python3 bench.py --mode $m --lz4-data $d --steps 3 --warmup 1 > $out/bench_${m}_$d.json 2> $out/bench_${m}_$d.err || { echo "$m $d failed"; tail -3 $out/bench_${m}_$d.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/bench_${m}_$d.json').read().strip().splitlines()[-1]); print('$m $d', d['value'], d['roofline']['kernel_avg_ms'], 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'])"
done; done
for m in ${MODES:-lz4 unlz4 unzstd}; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_$m -o run --output-format csv -- python3 bench.py --mode $m --lz4-data text --blocks 4096 --steps 2 --warmup 1 --no-cpu --verify 0 > $out/prof_$m.log 2>&1 || { echo "prof $m failed"; tail -3 $out/prof_$m.log; exit 1; }
done
echo suite done
