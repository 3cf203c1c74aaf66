bench.py --mode decrypt --total-gib 2048 --steps 3 --warmup 1
