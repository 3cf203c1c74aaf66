bench.py --mem host --steps 5 --warmup 1
