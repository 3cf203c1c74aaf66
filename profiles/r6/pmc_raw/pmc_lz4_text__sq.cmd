rocprofv3 --kernel-trace --pmc SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 --mode lz4 --blocks 4096
