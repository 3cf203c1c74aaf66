# per-task overheads of gcm_main_k on small blocks: as built, without the lane
# lift (bit-serial g_mul), without the per-task GHASH table build, without both
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ab_small
mkdir -p $out
for sz in 262144 65536; do
nb=$(( (8 << 30) / sz ))
for v in base LIFT GHBUILD LIFT2; do
  lib=juicefs_amd/libjfsx.so; [ $v != base ] && lib=juicefs_amd/_build/libjfsx_$v.so
  JFSX_LIB=$lib timeout -k 10 200 python3 bench.py --no-cpu --verify 0 --steps 5 --blocks $nb --block-bytes $sz > $out/$v.$sz.log 2>&1 || { echo "$v failed"; tail -3 $out/$v.$sz.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/$v.$sz.log').read().strip().splitlines()[-1]); print('$sz $v', d['value'], d['roofline']['kernel_avg_ms'])"
done
done
