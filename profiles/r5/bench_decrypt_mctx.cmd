bench.py --engine mctx --mode decrypt --steps 2 --warmup 1 --no-cpu
