bench.py --mode agg --threads 20 --steps 10 --no-cpu --agg-op seal --agg-max-mb 16
