bench.py --ragged --steps 10 --warmup 2
