# parity + timing for each build variant in juicefs_amd/_build (usage: bash scripts/gpu_variants.sh v1 v2 ...)
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in "$@"; do
  lib=juicefs_amd/_build/libjfsx_$v.so
  [ "$v" = "default" ] && lib=juicefs_amd/libjfsx.so
  JFSX_LIB=$lib timeout -k 10 300 python3 -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/var_${v}_pytest.log 2>&1
  rc=$?
  echo "$v pytest rc=$rc $(tail -1 gpurun_out/var_${v}_pytest.log)"
  [ $rc -le 1 ] || exit 1
  JFSX_LIB=$lib timeout -k 10 120 python3 bench.py --blocks 2048 --steps 5 --warmup 1 --no-cpu --verify 2 > gpurun_out/var_${v}_bench.log 2>&1 || { echo "$v bench failed"; tail -3 gpurun_out/var_${v}_bench.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/var_${v}_bench.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"
done
