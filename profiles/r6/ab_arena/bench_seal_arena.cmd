JFSX_PIPE_STATS=1 bench.py --mode agg --threads 20 --steps 10 --no-cpu --buffers heap --agg-crc seg --agg-op seal
