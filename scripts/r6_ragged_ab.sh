# per-object heap Encrypt on ragged 64 KiB-4 MiB blocks: small-group policy x keysetup stream
set -u
t=${1:-r6rg}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --no-cpu --warmup-seconds 3 --ragged --steps 20"
for rep in a b; do
  $S new_$rep $A || exit 1
  JFSX_AGG_INFLIGHT=64 $S oldpol_$rep $A || exit 1
  JFSX_KS_STREAM=0 $S noks_$rep $A || exit 1
  JFSX_AGG_INFLIGHT=64 JFSX_KS_STREAM=0 $S old_$rep $A || exit 1
done
