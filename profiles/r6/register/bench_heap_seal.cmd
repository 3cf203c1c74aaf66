bench.py --mode agg --buffers heap --agg-op seal --threads 20 --steps 10 --no-cpu
