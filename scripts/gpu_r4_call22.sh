# Round-4 call 22: GPU parity suite + smoke with the zstd parser's candidate
# extensions as the default (JFSX_ZC_WIN=287) and the shorter literal copy;
# A/B against the call-19 ZW287 build; then the zstd text line, its rocprof
# stats and PMC passes at 4096 objects.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4v || exit 1
out=gpurun_out/suite_r4v; mkdir -p $out
export TMPDIR=/tmp
ab() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 2 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
ab main && JFSX_LIB=juicefs_amd/_build/libjfsx_ZW287.so ab zw287 && ab main2 || exit 1
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQC="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
Z="--mode zstd --blocks 4096"
pmc zstd_text__fetch FETCH_SIZE $Z && pmc zstd_text__write WRITE_SIZE $Z && pmc zstd_text__sq "$SQC" $Z || exit 1
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_zstd_text -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 $Z --steps 2 --warmup 1 > $out/prof_zstd_text.log 2>&1 && echo "prof zstd ok" || exit 1
timeout -k 10 500 python3 bench.py $Z --steps 3 --warmup 1 > $out/bench_zstd_text.json 2> $out/bench_zstd_text.err && echo "zstd_text: $(tail -1 $out/bench_zstd_text.json | cut -c1-160)"
