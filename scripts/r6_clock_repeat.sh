# per-object heap Encrypt / Decrypt repeated in fresh processes with the GPU's DPM clock levels sampled
# over each run (bench.py --log-clocks): does the rare slow state follow a clock level?
set -u
t=${1:-r6ck}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --steps 10 --log-clocks"
for i in ${REPS:-1 2 3 4 5 6 7}; do
  $S seal_$i $A --agg-op seal || exit 1
  $S open_$i $A --agg-op open || exit 1
done
