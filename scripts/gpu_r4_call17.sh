# Round-4 call 17: GPU parity suite + smoke with the windowed zstd parser at 16 waves per CU (defaults), then the
# codec lines and PMC passes again (the LZ4 / zstd compressors changed).
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4q || exit 1
out=gpurun_out/suite_r4q; mkdir -p $out
export TMPDIR=/tmp
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQC="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
Z="--blocks 4096"
pmc zstd_text__fetch FETCH_SIZE --mode zstd $Z && pmc zstd_text__write WRITE_SIZE --mode zstd $Z && pmc zstd_text__sq "$SQC" --mode zstd --blocks 1024 && \
pmc lz4_text__fetch FETCH_SIZE --mode lz4 $Z && pmc lz4_text__write WRITE_SIZE --mode lz4 $Z && pmc lz4_text__sq "$SQC" --mode lz4 --blocks 1024 || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_zstd_text -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 --mode zstd $Z --steps 2 --warmup 1 > $out/prof_zstd_text.log 2>&1 && echo "prof zstd ok" && \
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_lz4_text -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 --mode lz4 $Z --steps 3 --warmup 1 > $out/prof_lz4_text.log 2>&1 && echo "prof lz4 ok" || exit 1
run() { local name=$1; shift; timeout -k 10 500 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-150)"; }
run lz4_text --mode lz4 $Z && run zstd_text --mode zstd $Z --steps 3 --warmup 1 && \
run aggcodec_lz4 --mode aggcodec --codec lz4 --threads 20 --steps 2 --warmup 1 && \
run aggcodec_zstd --mode aggcodec --codec zstd --threads 20 --steps 2 --warmup 1
