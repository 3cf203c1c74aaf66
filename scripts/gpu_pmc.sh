# HBM-traffic PMC passes (FETCH_SIZE / WRITE_SIZE, one counter per rocprofv3 run)
# on 4 GiB batches of each kernel; summary in gpurun_out/pmc_<tag>/pmc_summary.txt.
# usage: bash scripts/gpu_pmc.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$1
mkdir -p $out
export TMPDIR=/tmp
B="--blocks 1024 --steps 1 --warmup 0 --no-cpu --verify 0"
pmc() { name=$1; ctr=$2; shift 2; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py $B "$@" > $out/$name.log 2>&1 || { echo "$name failed"; grep -v "^ *@" $out/$name.log | tail -3; return 1; }; }
pmc gcm_fetch FETCH_SIZE && pmc gcm_write WRITE_SIZE && \
pmc gcmbs_fetch FETCH_SIZE --aes bitslice && pmc gcmbs_write WRITE_SIZE --aes bitslice && \
pmc cp_fetch FETCH_SIZE --algo chacha20poly1305 && pmc cp_write WRITE_SIZE --algo chacha20poly1305 && \
pmc crc_fetch FETCH_SIZE --mode crc && \
pmc gcm_lds "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_INSTS_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo pmc done
