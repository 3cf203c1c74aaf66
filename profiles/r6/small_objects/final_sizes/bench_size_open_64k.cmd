bench.py --mode agg --threads 20 --buffers heap --agg-op open --agg-crc seg --block-bytes 65536 --steps 400
