# Round 2 counters: VALU issue rates, compute/stall counters of gcm_main_k and
# cp_main_k (4 GiB batches), and the 64 GiB FETCH/WRITE passes that crashed in
# round 1 (now with the one-launch generator).  usage: bash scripts/gpu_r2_pmc.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/pmc_$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 120 ./tools/valu_rates > $out/valu_rates.txt 2>&1 || { echo valu_rates failed; exit 1; }
cat $out/valu_rates.txt
timeout -k 10 60 rocprofv3 -L > $out/counters_list.txt 2>&1 || true
B="--blocks 1024 --steps 1 --warmup 0 --no-cpu --verify 0"
pmc() { name=$1; ctr=$2; shift 2; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py "$@" > $out/$name.log 2>&1 || { echo "$name failed rc=$?"; grep -v "^ *@" $out/$name.log | tail -5; return 1; }; }
pmc gcm_a "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE" $B && \
pmc gcm_b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" $B && \
pmc cp_a "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE" $B --algo chacha20poly1305 && \
pmc cp_b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" $B --algo chacha20poly1305 && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo "4 GiB passes done" && \
pmc gcm64_fetch FETCH_SIZE --blocks 16384 --steps 1 --warmup 0 --no-cpu --verify 0 && \
pmc gcm64_write WRITE_SIZE --blocks 16384 --steps 1 --warmup 0 --no-cpu --verify 0 && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo "pmc done"
