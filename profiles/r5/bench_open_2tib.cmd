bench.py --mode open --total-gib 2048 --steps 3 --warmup 1
