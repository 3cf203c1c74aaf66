# Round-4 call 11: zstd compressor section stamps (diagnostic build
# JFSX_ZC_STAMP: waves 0-1 print parse / entropy wall-clock ticks per object),
# at 512 and 4096 objects of text.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4k; mkdir -p $out
export TMPDIR=/tmp
for nb in 512 4096; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_ZSTAMP.so timeout -k 10 300 python3 bench.py --mode zstd --blocks $nb --steps 1 --warmup 0 --no-cpu --verify 0 > $out/stamp_$nb.log 2>&1 || { echo "stamp $nb failed"; tail -5 $out/stamp_$nb.log; exit 1; }
  grep "zc-stamp" $out/stamp_$nb.log | head -8
done
# the register-window parser (JFSX_ZC_WIN=1): parity, then A/B against the default
JFSX_LIB=juicefs_amd/_build/libjfsx_ZWIN.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zstdc.py tests/test_compress_contract.py -x -q --timeout 120 --timeout-method thread > $out/zwin_pytest.log 2>&1 || { echo "ZWIN parity failed"; tail -30 $out/zwin_pytest.log; exit 1; }
echo "ZWIN parity: $(tail -1 $out/zwin_pytest.log)"
ab() {
  name=$1; lib=$2
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode zstd --blocks 4096 --steps 2 --warmup 1 --no-cpu --verify 4 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -5 $out/ab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/ab_$name.json').read().splitlines()[-1]); print('%-6s value %7.3f kernel_ms %9.1f' % ('$name', d['value'], d['roofline']['kernel_avg_ms']))"
}
ab base juicefs_amd/libjfsx.so && ab zwin juicefs_amd/_build/libjfsx_ZWIN.so && ab base2 juicefs_amd/libjfsx.so && ab zwin2 juicefs_amd/_build/libjfsx_ZWIN.so
