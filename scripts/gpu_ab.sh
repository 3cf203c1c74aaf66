# Same-box A/B of build variants: parity on each variant, then interleaved
# timing reps.  usage: bash scripts/gpu_ab.sh <tag> "<bench args>" name=lib ...
# (lib "default" = juicefs_amd/libjfsx.so, else juicefs_amd/_build/libjfsx_<lib>.so)
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1; args=$2; shift 2
out=gpurun_out/ab_$tag
mkdir -p $out
for spec in "$@"; do
  name=${spec%%=*}; v=${spec#*=}
  lib=juicefs_amd/_build/libjfsx_$v.so; [ "$v" = default ] && lib=juicefs_amd/libjfsx.so
  JFSX_LIB=$lib timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -x -q -m gpu --timeout 120 --timeout-method thread > $out/$name.pytest.log 2>&1 && grep -q passed $out/$name.pytest.log && ! grep -q skipped $out/$name.pytest.log || { echo "$name parity FAILED"; tail -5 $out/$name.pytest.log; exit 1; }
  echo "$name parity: $(tail -1 $out/$name.pytest.log)"
done
for rep in ${AB_REPS:-1 2 3}; do
  for spec in "$@"; do
    name=${spec%%=*}; v=${spec#*=}
    lib=juicefs_amd/_build/libjfsx_$v.so; [ "$v" = default ] && lib=juicefs_amd/libjfsx.so
    JFSX_LIB=$lib timeout -k 10 200 python3 bench.py $args --no-cpu --verify 2 > $out/$name.$rep.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.$rep.log; exit 1; }
    python3 -c "import json; d=json.loads(open('$out/$name.$rep.log').read().strip().splitlines()[-1]); print('$name', d['value'], d['roofline']['kernel_avg_ms'])"
  done
done
