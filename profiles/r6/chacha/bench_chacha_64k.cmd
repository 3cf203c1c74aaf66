bench.py --mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --algo chacha20poly1305 --block-bytes 65536 --steps 400
