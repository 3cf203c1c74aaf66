# Round 3: the zstd compressor with the lane-0 entropy build (probe + the
# whole GPU suite on that library), CRC-verify A/B (64-B lane spans vs 16-B
# rows), and last a printf-traced run of the wave entropy build on the input
# that hung (its last printed stage locates the hang).
# usage: bash scripts/gpu_r3c.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
L0=juicefs_amd/_build/libjfsx_ZCLANE0.so
JFSX_LIB=$L0 timeout -k 10 240 python3 -u scripts/zstdc_probe.py 4194304 > $out/zc_lane0.txt 2>&1
rc=$?; echo "lane0 probe rc=$rc"; tail -3 $out/zc_lane0.txt
[ $rc -eq 0 ] || exit 1
JFSX_LIB=$L0 timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error' $out/pytest.log | head -20; exit 1; }
for v in new old new old; do
  lib=$L0; [ $v = old ] && lib=juicefs_amd/_build/libjfsx_CRC16.so
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode crc --no-cpu --steps 10 > $out/crc_$v.json 2> $out/crc_$v.err || { echo "crc $v failed"; tail -3 $out/crc_$v.err; exit 1; }
  echo "crc $v: $(python3 -c "import json,sys; d=json.loads(open('$out/crc_$v.json').read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])")"
done
for v in 3 4 6 3; do
  lib=$L0; [ $v != 3 ] && lib=juicefs_amd/_build/libjfsx_RING$v.so
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mem host --blocks 1024 --steps 6 --warmup 1 --no-cpu > $out/ingest_ring$v.json 2> $out/ingest_ring$v.err || { echo "ingest $v failed"; tail -3 $out/ingest_ring$v.err; exit 1; }
  echo "ingest ring $v: $(python3 -c "import json,sys; d=json.loads(open('$out/ingest_ring$v.json').read().splitlines()[-1]); print(d['value'], d['roofline']['pcie_measured'], d['roofline']['frac'])")"
done
JFSX_LIB=juicefs_amd/_build/libjfsx_ZCTRACE.so timeout -k 5 40 python3 -u -c "
from juicefs_amd import engine as E
e = E.Engine(0)
print(len(e.zstd_compress([b'zstd' * 100])[0]), flush=True)
" > $out/zc_trace.txt 2>&1
echo "trace rc=$?"; tail -30 $out/zc_trace.txt
