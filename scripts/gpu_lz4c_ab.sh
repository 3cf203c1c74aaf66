# LZ4 compressor A/B: GPU parity (default build), then compress bench lines
# (text / random, 16 GiB) for each library variant.
# usage: bash scripts/gpu_lz4c_ab.sh <tag> name=lib ...
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/lz4cab_$tag
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_lz4.py -x -v -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $out/pytest.log | head -20; exit 1; }
for data in text random; do
  for spec in "$@"; do
    name=${spec%%=*}; v=${spec#*=}
    lib=juicefs_amd/_build/libjfsx_$v.so; [ "$v" = default ] && lib=juicefs_amd/libjfsx.so
    JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --mode lz4 --lz4-data $data --blocks 4096 --steps 2 --warmup 1 --no-cpu --verify 4 > $out/$name.$data.log 2>&1 || { echo "$name $data failed"; tail -3 $out/$name.$data.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/$name.$data.log').read().strip().splitlines()[-1]); print('$name $data', d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
