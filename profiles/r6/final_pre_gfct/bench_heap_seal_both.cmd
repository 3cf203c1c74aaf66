bench.py --mode agg --threads 20 --steps 10 --buffers heap --agg-op seal --agg-crc both
