bench.py --mode agg --threads 20 --steps 5 --warmup 1 --no-cpu
