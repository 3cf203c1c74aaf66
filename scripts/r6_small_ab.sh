# A/B of the aggregator's small-group policy (JFSX_AGG_INFLIGHT: 2 = new
# default, 64 = the old "go whenever the engine is busy") on per-object heap
# Encrypt at 64 KiB, 256 KiB, 1 MiB and 4 MiB, no CPU leg.
set -u
t=${1:-r6u}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --no-cpu --warmup-seconds 3"
for sz in 65536:400 262144:100 1048576:30 4194304:10; do
  b=${sz%%:*}; n=${sz##*:}
  JFSX_PIPE_STATS=1 $S new_$b $A --block-bytes $b --steps $n || exit 1
  JFSX_PIPE_STATS=1 JFSX_AGG_INFLIGHT=64 $S old_$b $A --block-bytes $b --steps $n || exit 1
done
