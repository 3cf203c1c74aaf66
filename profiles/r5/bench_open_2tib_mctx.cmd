bench.py --engine mctx --mode open --total-gib 2048 --steps 3 --warmup 1 --no-cpu
