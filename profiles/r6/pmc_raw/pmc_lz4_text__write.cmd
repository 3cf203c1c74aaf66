rocprofv3 --kernel-trace --pmc WRITE_SIZE -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 --mode lz4 --blocks 4096
