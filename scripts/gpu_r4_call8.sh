# Round-4 call 8: LZ4 compressor speculation width (JFSX_LZ4_K0: probes of the
# first search step, doubling on each step without a match): parity of each
# build on the LZ4-library byte-for-byte tests, then a same-box A/B at 16 GiB
# of text (K0 = 64 is the round-3 kernel).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4h; mkdir -p $out
export TMPDIR=/tmp
B=juicefs_amd/_build
for k in 4 8 16; do
  JFSX_LIB=$B/libjfsx_LK$k.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lz4.py tests/test_compress_contract.py -x -q --timeout 120 --timeout-method thread > $out/lk${k}_pytest.log 2>&1 || { echo "LK$k parity failed"; tail -20 $out/lk${k}_pytest.log; exit 1; }
  echo "LK$k parity: $(tail -1 $out/lk${k}_pytest.log)"
done
ab() {
  name=$1; lib=$2
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode lz4 --blocks 4096 --steps 3 --warmup 1 --no-cpu --verify 4 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -5 $out/ab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/ab_$name.json').read().splitlines()[-1]); print('%-6s value %7.3f kernel_ms %9.1f' % ('$name', d['value'], d['roofline']['kernel_avg_ms']))"
}
ab k64 juicefs_amd/libjfsx.so && ab k4 $B/libjfsx_LK4.so && ab k8 $B/libjfsx_LK8.so && ab k16 $B/libjfsx_LK16.so && ab k8b $B/libjfsx_LK8.so
