# pipelined-group fill (JFSX_AGG_FILL_MB 4 / 12) on per-object heap Decrypt and Encrypt, 4 MiB blocks,
# 20 callers, fresh process per run, alternating on one box
set -u
t=${1:-r6fl}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --steps 10"
for rep in 1 2 3 4; do
  for f in 4 12; do
    JFSX_AGG_FILL_MB=$f $S open_f${f}_$rep $A --agg-op open || exit 1
    JFSX_AGG_FILL_MB=$f $S seal_f${f}_$rep $A --agg-op seal || exit 1
  done
done
