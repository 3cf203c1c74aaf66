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
# GCM: 12 waves (3 per SIMD, 168 VGPRs) with 2 or 3 T-table rows per iteration
# against the 16-wave default (parity first on the 3-row build)
JFSX_LIB=juicefs_amd/_build/libjfsx_W12U3.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -x -q --timeout 120 --timeout-method thread > $out/w12u3_pytest.log 2>&1 || { echo "W12U3 parity failed"; tail -20 $out/w12u3_pytest.log; exit 1; }
echo "W12U3 parity: $(tail -1 $out/w12u3_pytest.log)"
gab() {
  name=$1; lib=$2
  JFSX_LIB=$lib timeout -k 10 200 python3 bench.py --blocks 4096 --steps 5 --warmup 1 --no-cpu --verify 0 > $out/gab_$name.json 2> $out/gab_$name.err || { echo "$name failed"; tail -5 $out/gab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/gab_$name.json').read().splitlines()[-1]); print('%-8s value %8.2f kernel_ms %7.3f' % ('$name', d['value'], d['roofline']['kernel_avg_ms']))"
}
B=juicefs_amd/_build
gab base1 juicefs_amd/libjfsx.so && gab w12u3 $B/libjfsx_W12U3.so && gab w12u2 $B/libjfsx_W12U2.so && \
gab base2 juicefs_amd/libjfsx.so && gab w12u3b $B/libjfsx_W12U3.so
