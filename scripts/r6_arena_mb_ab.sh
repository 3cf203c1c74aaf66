# shared staging arena size (JFSX_AGG_ARENA_MB 32 / 64 / 128) on per-object heap Encrypt and Decrypt,
# 4 MiB, 20 callers, no CPU leg, alternating on one box
set -u
t=${1:-r6am}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --steps 10"
for rep in a b; do
  for m in 32 64 128; do
    JFSX_AGG_ARENA_MB=$m $S seal_${m}_$rep $A --agg-op seal || exit 1
    JFSX_AGG_ARENA_MB=$m $S open_${m}_$rep $A --agg-op open || exit 1
  done
done
