# Round-4 call 39: non-temporal block streams in the GCM and CRC-verify
# kernels -- GPU suite + smoke, then the configs[1] / [3] / [4]-GCM lines and
# the CRC verify line with same-run CPU baselines and full checks, their
# rocprof stats, and PMC traffic / SQ passes.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4j2 || exit 1
out=gpurun_out/suite_r4j2; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-110)"; }
run seal_gcm && run open_gcm --mode open && run crc_verify --mode crc && run seal_gcm_ragged --ragged && run open_gcm_ragged --ragged --mode open || exit 1
prof() { local name=$1; shift; timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$name -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 "$@" > $out/prof_$name.log 2>&1 && echo "prof $name ok"; }
prof gcm --steps 10 --warmup 2 && prof open_gcm --mode open --steps 10 --warmup 2 && prof crc --mode crc --steps 10 --warmup 2 && prof gcm_ragged --ragged --steps 10 --warmup 2 || exit 1
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQ="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
pmc seal_gcm__fetch FETCH_SIZE && pmc seal_gcm__write WRITE_SIZE && pmc crc_verify__fetch FETCH_SIZE --mode crc && pmc crc_verify__write WRITE_SIZE --mode crc && \
pmc open_gcm__fetch FETCH_SIZE --mode open && pmc open_gcm__write WRITE_SIZE --mode open && \
pmc seal_gcm__sq "$SQ" --blocks 1024 && pmc crc_verify__sq "$SQ" --blocks 1024 --mode crc && pmc open_gcm__sq "$SQ" --blocks 1024 --mode open
