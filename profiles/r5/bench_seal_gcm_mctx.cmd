bench.py --engine mctx --steps 10 --warmup 2
