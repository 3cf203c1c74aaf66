bench.py --mode agg --buffers heap --agg-op open --threads 20 --steps 10 --no-cpu
