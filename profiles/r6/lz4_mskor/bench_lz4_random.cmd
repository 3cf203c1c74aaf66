bench.py --mode lz4 --lz4-data random --blocks 4096 --steps 5 --warmup 1
