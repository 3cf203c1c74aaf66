bench.py --mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --steps 10 --agg-op seal
