bench.py --mem host --total-gib 256 --steps 3 --warmup 1
