bench.py --mode agg --agg-op seal --agg-max-mb 16 --threads 20 --steps 10 --no-cpu
