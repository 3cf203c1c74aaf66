rocprofv3 --kernel-trace --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 --blocks 1024
