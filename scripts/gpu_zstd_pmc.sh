# zstd decoder instruction mix (PMC) on a 4 GiB text batch for one library.
# usage: bash scripts/gpu_lz4_pmc2.sh <tag> <lib>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/zstdpmc_$1
mkdir -p $out
export TMPDIR=/tmp
export JFSX_LIB=$2
B="--blocks ${BLOCKS:-1024} --steps 1 --warmup 0 --no-cpu --verify 0 --lz4-data text --mode unzstd"
pmc() { name=$1; ctr=$2; shift 2; timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py "$@" > $out/$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/$name.log | tail -3; return 1; }; }
pmc d_a "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY GRBM_GUI_ACTIVE" $B && \
pmc d_b "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" $B && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo pmc done && grep -A20 zstd_decompress $out/pmc_summary.txt
