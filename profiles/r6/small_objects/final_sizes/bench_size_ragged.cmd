bench.py --mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --ragged --steps 20
