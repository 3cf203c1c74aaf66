bench.py --mode agg --agg-op verify --threads 20 --steps 10 --no-cpu
