bench.py --steps 10 --warmup 2 --no-cpu
