# Round-4 call 6: the zstd compressor's object assignment A/B (ticket queue,
# waves per CU) after a parity pass on the queue; the per-call zstd lines through
# the aggregator; host ingest with the PCIe probe before and after the ring.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4f; mkdir -p $out
export TMPDIR=/tmp
JFSX_ZC_QUEUE=1 JFSX_ZC_WAVES=11 timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zstdc.py -x -q --timeout 120 --timeout-method thread > $out/zcq_pytest.log 2>&1 || { echo "queue parity failed"; tail -20 $out/zcq_pytest.log; exit 1; }
echo "zstd compressor ticket queue parity: $(tail -1 $out/zcq_pytest.log)"
ab() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --mode zstd --blocks 4096 --steps 2 --warmup 1 --no-cpu --verify 2 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -5 $out/ab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/ab_$name.json').read().splitlines()[-1]); print('%-8s %s value %8.3f kernel_ms %9.1f' % ('$name', '$*', d['value'], d['roofline']['kernel_avg_ms']))"
}
ab w8 JFSX_ZC_WAVES=8 && ab w11 JFSX_ZC_WAVES=11 && ab w8q JFSX_ZC_WAVES=8 JFSX_ZC_QUEUE=1 && ab w11q JFSX_ZC_WAVES=11 JFSX_ZC_QUEUE=1 || exit 1
bash scripts/gpu_r4_suite.sh r4f agg_codec_zstd
s=gpurun_out/suite_r4f
timeout -k 10 500 python3 bench.py --mem host --blocks 2048 --steps 8 --warmup 1 > $s/bench_ingest_gcm.json 2> $s/bench_ingest_gcm.err || { echo "ingest failed"; tail -5 $s/bench_ingest_gcm.err; exit 1; }
echo "ingest: $(tail -1 $s/bench_ingest_gcm.json | cut -c1-160)"
