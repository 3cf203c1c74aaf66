# LZ4 stage: GPU tests (LZ4 parity + aggregator paths) and the four 64 GiB
# bench lines with CPU baselines.  usage: bash scripts/gpu_lz4_check.sh <tag> [bench]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/lz4chk_$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 500 python3 -u -m pytest tests/test_gpu_lz4.py tests/test_gpu_agg.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $out/pytest.log | head -20; exit 1; }
[ "${2:-}" = bench ] || exit 0
for m in unlz4 lz4; do for d in text random; do
  timeout -k 10 400 python3 bench.py --mode $m --lz4-data $d --steps 3 --warmup 1 > $out/bench_${m}_$d.json 2> $out/bench_${m}_$d.err || { echo "$m $d failed"; tail -3 $out/bench_${m}_$d.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/bench_${m}_$d.json').read().strip().splitlines()[-1]); print('$m $d', d['value'], d['roofline']['kernel_avg_ms'], 'cpu', d['cpu_baseline'] and d['cpu_baseline']['value'])"
done; done
