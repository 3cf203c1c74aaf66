bench.py --mode agg --threads 20 --steps 10 --agg-op seal --agg-max-mb 16
