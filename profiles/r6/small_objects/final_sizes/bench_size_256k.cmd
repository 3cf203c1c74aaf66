bench.py --mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --block-bytes 262144 --steps 100
