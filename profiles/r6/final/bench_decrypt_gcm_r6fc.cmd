bench.py --mode decrypt --steps 5 --warmup 1
