rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --verify 0 --mode lz4 --blocks 4096 --steps 3 --warmup 1
