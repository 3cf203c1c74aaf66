rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --verify 0 --mode decrypt --steps 5 --warmup 1
