bench.py --mode agg --agg-op checksum --threads 20 --steps 10 --no-cpu
