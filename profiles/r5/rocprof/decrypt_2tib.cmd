rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --verify 0 --mode decrypt --total-gib 2048 --steps 2 --warmup 1
