# Round-4 call 9: zstd compressor, narrow steps compare hashes by readlane
# instead of hashLog x 2 ballots (ZK4R / ZK8R) against ZK4: parity, then A/B.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4i; mkdir -p $out
export TMPDIR=/tmp
B=juicefs_amd/_build
for v in ZK4R ZK8R; do
  JFSX_LIB=$B/libjfsx_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_zstdc.py tests/test_compress_contract.py -x -q --timeout 120 --timeout-method thread > $out/${v}_pytest.log 2>&1 || { echo "$v parity failed"; tail -20 $out/${v}_pytest.log; exit 1; }
  echo "$v parity: $(tail -1 $out/${v}_pytest.log)"
done
ab() {
  name=$1; lib=$2
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode zstd --blocks 4096 --steps 2 --warmup 1 --no-cpu --verify 4 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -5 $out/ab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/ab_$name.json').read().splitlines()[-1]); print('%-6s value %7.3f kernel_ms %9.1f' % ('$name', d['value'], d['roofline']['kernel_avg_ms']))"
}
ab zk4 $B/libjfsx_ZK4.so && ab zk4r $B/libjfsx_ZK4R.so && ab zk8r $B/libjfsx_ZK8R.so && ab zk4rb $B/libjfsx_ZK4R.so
