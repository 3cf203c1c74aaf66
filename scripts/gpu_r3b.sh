# Round 3, second contact: table-lookup probe, the GPU suite without the zstd
# compressor, CRC-verify A/B (64-B lane spans vs 16-B rows), then the zstd
# compressor one object per call: lane-0 entropy build first, wave entropy
# (the default, suspected of hanging) last.   usage: bash scripts/gpu_r3b.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/gather_probe > $out/gather_probe.txt 2>&1 || { echo "gather_probe failed"; exit 1; }
cat $out/gather_probe.txt
timeout -k 10 900 python3 -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread \
  --ignore=tests/test_gpu_zstdc.py --ignore=tests/test_compress_contract.py > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error' $out/pytest.log | head -20; exit 1; }
for v in new old new old; do
  lib=""; [ $v = old ] && lib=juicefs_amd/_build/libjfsx_CRC16.so
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode crc --no-cpu --steps 10 > $out/crc_$v.json 2> $out/crc_$v.err || { echo "crc $v failed"; tail -3 $out/crc_$v.err; exit 1; }
  echo "crc $v: $(python3 -c "import json,sys; d=json.loads(open('$out/crc_$v.json').read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])")"
done
JFSX_LIB=juicefs_amd/_build/libjfsx_ZCLANE0.so timeout -k 10 240 python3 -u scripts/zstdc_probe.py 4194304 > $out/zc_lane0.txt 2>&1
echo "lane0 probe rc=$?"; tail -3 $out/zc_lane0.txt
timeout -k 10 120 python3 -u scripts/zstdc_probe.py 4194304 > $out/zc_wave.txt 2>&1
echo "wave probe rc=$?"; tail -3 $out/zc_wave.txt
