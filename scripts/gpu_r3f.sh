# Round 3: CRC-verify kernel variants (lane chunk 64 / 128 B, waves per SIMD),
# each checked by the GPU CRC tests on its own library, then timed in
# alternation.  usage: bash scripts/gpu_r3f.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
for v in S128 S128W4 S64W6; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_CRC$v.so timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_object_checksum.py tests/test_gpu_parity.py -k "crc or checksum or CRC" > $out/pytest_$v.log 2>&1 || { echo "$v tests failed"; tail -5 $out/pytest_$v.log; exit 1; }
  echo "$v tests: $(tail -1 $out/pytest_$v.log)"
done
for rep in 1 2; do
for v in base S128 S128W4 S64W6; do
  lib=""; [ $v != base ] && lib=juicefs_amd/_build/libjfsx_CRC$v.so
  JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode crc --no-cpu --steps 10 > $out/crc_$v.$rep.json 2> $out/crc_$v.$rep.err || { echo "crc $v failed"; tail -3 $out/crc_$v.$rep.err; exit 1; }
  echo "crc $v.$rep: $(python3 -c "import json,sys; d=json.loads(open('$out/crc_$v.$rep.json').read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'], d['roofline']['frac'])")"
done
done
