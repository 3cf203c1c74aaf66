# Zstandard decoder A/B: GPU parity of the default build, section stamps of a
# -DJFSX_ZSTD_STAMP variant (if built), then text decompress bench lines
# (16 GiB) for each library variant on the same box.
# usage: bash scripts/gpu_zstd_ab.sh <tag> name=lib ...
# (lib "default" = juicefs_amd/libjfsx.so, else juicefs_amd/_build/libjfsx_<lib>.so)
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/zstdab_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zstd.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -3 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $out/pytest.log | head -20; exit 1; }
if [ -f juicefs_amd/_build/libjfsx_ZSTAMP.so ]; then
  JFSX_LIB=juicefs_amd/_build/libjfsx_ZSTAMP.so timeout -k 10 300 python3 scripts/zstd_stamps.py 256 > $out/stamps.log 2>&1 || { tail -3 $out/stamps.log; exit 1; }
  cat $out/stamps.log
fi
for rep in ${REPS:-1 2}; do
  for spec in "$@"; do
    name=${spec%%=*}; v=${spec#*=}
    lib=juicefs_amd/_build/libjfsx_$v.so; [ "$v" = default ] && lib=juicefs_amd/libjfsx.so
    JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode unzstd --lz4-data text --blocks ${BLOCKS:-3584} --steps 2 --warmup 1 --no-cpu --verify 4 > $out/$name.$rep.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/$name.$rep.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
