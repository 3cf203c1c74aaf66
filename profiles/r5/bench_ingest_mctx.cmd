bench.py --engine mctx --mem host --steps 2 --warmup 1 --no-cpu
