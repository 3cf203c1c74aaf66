# Round-4 call 29: GPU parity suite + smoke on the current build, then the
# zstd compressor lines (text, random; same-run libzstd baselines), its
# rocprof stats and PMC passes at 4096 objects.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4g2 || exit 1
out=gpurun_out/suite_r4g2; mkdir -p $out
export TMPDIR=/tmp
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQC="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
Z="--mode zstd --blocks 4096"
pmc zstd_text__fetch FETCH_SIZE $Z && pmc zstd_text__write WRITE_SIZE $Z && pmc zstd_text__sq "$SQC" $Z || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_zstd_text -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 $Z --steps 2 --warmup 1 > $out/prof_zstd_text.log 2>&1 && echo "prof zstd ok" || exit 1
run() { local name=$1; shift; timeout -k 10 500 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-150)"; }
run zstd_text $Z --steps 3 --warmup 1 && run zstd_random $Z --lz4-data random --steps 3 --warmup 1
