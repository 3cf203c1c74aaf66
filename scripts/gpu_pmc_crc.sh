# Stall-breakdown PMC passes for the CRC-only kernel (crc_segments_k), 4 GiB batch.
# usage: bash scripts/gpu_pmc_crc.sh <tag> [extra bench args]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmccrc_$1
shift
EXTRA=("$@")
mkdir -p $out
export TMPDIR=/tmp
B="--mode crc --blocks 1024 --steps 1 --warmup 0 --no-cpu --verify 0"
pmc() { name=$1; ctr=$2; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py $B "${EXTRA[@]}" > $out/$name.log 2>&1 || { echo "$name failed"; grep -v "^ *@" $out/$name.log | tail -3; return 1; }; }
pmc lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" && \
pmc wait "SQ_WAIT_INST_LDS SQ_WAIT_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_WAIT_INST_ANY SQ_INSTS_SALU" && \
pmc fetch FETCH_SIZE && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && grep -A12 crc_segments $out/pmc_summary.txt
