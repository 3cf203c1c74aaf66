# aggregator batch cap (--agg-max-mb 12 / 16 / 24) on per-object heap Encrypt and Decrypt, 4 MiB, no CPU leg
set -u
t=${1:-r6mm}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --steps 10"
for rep in a b; do
  for m in 12 16 24; do
    JFSX_PIPE_STATS=1 $S seal_${m}_$rep $A --agg-op seal --agg-max-mb $m || exit 1
  done
done
for m in 12 16 24; do $S open_${m} $A --agg-op open --agg-max-mb $m || exit 1; done
