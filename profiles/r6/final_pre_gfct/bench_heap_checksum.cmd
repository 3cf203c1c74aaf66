bench.py --mode agg --threads 20 --steps 10 --agg-op checksum
