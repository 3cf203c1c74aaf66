bench.py --mode lz4 --blocks 4096 --steps 5 --warmup 1
