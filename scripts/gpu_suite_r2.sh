# Round-2 measurement suite on the final tree: bench lines for every config and
# mode, rocprofv3 kernel stats, 64 GiB HBM-traffic PMC passes, compute counters.
# usage: bash scripts/gpu_suite_r2.sh <tag>      (results under gpurun_out/suite_<tag>)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_$1
mkdir -p $out
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 400 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-150)"; }
prof() { name=$1; shift; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_$name -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --verify 0 "$@" > $out/prof_$name.log 2>&1 || { echo "prof $name failed"; tail -5 $out/prof_$name.log; return 1; }; }
pmc() { name=$1; ctr=$2; shift 2; timeout -s KILL 150 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/$name.log | tail -3; return 1; }; }
run seal_gcm && \
run seal_gcm_bitslice --aes bitslice --no-cpu && \
run seal_chacha --algo chacha20poly1305 --no-cpu && \
run open_gcm --mode open --no-cpu && \
run open_chacha --mode open --algo chacha20poly1305 --no-cpu && \
run crc_verify --mode crc --no-cpu && \
run seal_gcm_ragged --ragged --no-cpu && run open_gcm_ragged --ragged --mode open --no-cpu && \
run seal_chacha_ragged --ragged --algo chacha20poly1305 --no-cpu && run open_chacha_ragged --ragged --mode open --algo chacha20poly1305 --no-cpu && \
run decrypt_gcm --mode decrypt --no-cpu && \
run ingest_gcm --mem host --blocks 2048 --steps 8 --warmup 1 --no-cpu && \
prof gcm && prof gcm_ragged --ragged && prof cp --algo chacha20poly1305 && prof crc --mode crc && \
pmc gcm_fetch FETCH_SIZE && pmc gcm_write WRITE_SIZE && \
pmc gcmbs_fetch FETCH_SIZE --aes bitslice && pmc gcmbs_write WRITE_SIZE --aes bitslice && \
pmc cp_fetch FETCH_SIZE --algo chacha20poly1305 && pmc cp_write WRITE_SIZE --algo chacha20poly1305 && \
pmc crc_fetch FETCH_SIZE --mode crc && \
python3 scripts/pmc_traffic.py $out 64 > $out/pmc_traffic.json && \
pmc gcm_a "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE" --blocks 1024 && \
pmc gcm_b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" --blocks 1024 && \
pmc cp_a "SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_INSTS_LDS GRBM_GUI_ACTIVE" --blocks 1024 --algo chacha20poly1305 && \
pmc cp_b "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_ANY SQ_INSTS_SALU GRBM_GUI_ACTIVE" --blocks 1024 --algo chacha20poly1305 && \
echo suite done
