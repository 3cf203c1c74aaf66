# per-object heap Decrypt repeated in fresh processes with the pipeline's
# stage timings (JFSX_PIPE_STATS): what differs in a slow run
set -u
t=${1:-r6or}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --steps 10 --agg-op open"
for i in 1 2 3 4 5 6 7 8; do JFSX_PIPE_STATS=1 $S open_$i $A || exit 1; done
