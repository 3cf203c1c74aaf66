bench.py --mode agg --buffers heap --agg-op seal --threads 20 --steps 3 --no-cpu --warmup-seconds 2
