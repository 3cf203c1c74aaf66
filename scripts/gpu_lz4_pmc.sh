# LZ4 compressor / decompressor instruction mix (PMC) on a 4 GiB text batch.
# usage: bash scripts/gpu_lz4_pmc.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/lz4pmc_$1
mkdir -p $out
export TMPDIR=/tmp
B="--blocks 1024 --steps 1 --warmup 0 --no-cpu --verify 0 --lz4-data text"
pmc() { name=$1; ctr=$2; shift 2; timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py "$@" > $out/$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/$name.log | tail -3; return 1; }; }
pmc c_a "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" $B --mode lz4 && \
pmc c_b "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" $B --mode lz4 && \
pmc d_a "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" $B --mode unlz4 && \
pmc d_b "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE" $B --mode unlz4 && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo pmc done
