# GPU tests, then one-segment tasks for small batches (default) vs the 64 KiB minimum
# (JFSX_GCM_SEG_TASKS=0) on per-object heap Encrypt by block size (no CPU leg)
set -u
t=${1:-r6st}
S="bash scripts/suite.sh $t"
A="--mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --no-cpu --warmup-seconds 3"
$S tests || exit 1
for sz in 65536:400 262144:100 1048576:30 4194304:10; do
  b=${sz%%:*}; n=${sz##*:}
  $S line seg_$b $A --block-bytes $b --steps $n || exit 1
  JFSX_GCM_SEG_TASKS=0 $S line min64_$b $A --block-bytes $b --steps $n || exit 1
done
$S line seg_ragged $A --ragged --steps 20 || exit 1
JFSX_GCM_SEG_TASKS=0 $S line min64_ragged $A --ragged --steps 20
