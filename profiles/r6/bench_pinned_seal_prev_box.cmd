bench.py --mode agg --agg-op seal --threads 20 --steps 5 --no-cpu --agg-max-mb 16
