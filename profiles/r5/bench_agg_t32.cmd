bench.py --mode agg --threads 32 --steps 5 --warmup 1 --no-cpu
