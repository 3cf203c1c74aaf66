bench.py --mode agg --agg-op open --threads 20 --steps 5 --warmup 1
