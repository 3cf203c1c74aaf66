# A/B of the working tree's libjfsx.so against juicefs_amd/_build/libjfsx_prev.so
# (the previous commit) on one box.  usage: bash scripts/gpu_ab_prev.sh <tag> [bench args...]
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1; shift
out=gpurun_out/ab_$tag
mkdir -p $out
for rep in 1 2; do
for v in prev new; do
  lib=juicefs_amd/libjfsx.so; [ $v = prev ] && lib=juicefs_amd/_build/libjfsx_prev.so
  JFSX_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --verify 2 "$@" > $out/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $out/$v.$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/$v.$rep.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"
done
done
