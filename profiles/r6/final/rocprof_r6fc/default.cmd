rocprofv3 --kernel-trace --stats -- python3 bench.py --no-cpu --verify 0 
