bench.py --mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --block-bytes 65536 --steps 400
