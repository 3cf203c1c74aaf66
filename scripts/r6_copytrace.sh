# per-object heap Decrypt / Encrypt in fresh processes under rocprofv3 --memory-copy-trace (no counters):
# per-copy durations of fast and slow runs
set -u
t=${1:-r6mc}
out=gpurun_out/suite_$t
mkdir -p $out
export TMPDIR=/tmp
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 2 --steps 5"
for i in 1 2 3 4 5 6 7 8; do
  for op in open seal; do
    timeout -k 10 150 rocprofv3 --memory-copy-trace -d $out/${op}_$i -o run --output-format csv \
      -- python3 bench.py $A --agg-op $op > $out/${op}_$i.log 2>&1 || { echo "$op $i failed"; tail -3 $out/${op}_$i.log; exit 1; }
    echo "$op $i: $(grep '^{' $out/${op}_$i.log | tail -1 | cut -c1-120)"
  done
done
