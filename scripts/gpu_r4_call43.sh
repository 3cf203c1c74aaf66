# Round-4 call 43: gcm_finalize_k's lifts by nibble-table products (FN1)
# against the bit-serial g_mul (main): parity on FN1, the configs[1] / [3]
# step A/B and the finalize kernel's rocprof time, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ai; mkdir -p $out
export TMPDIR=/tmp
F=juicefs_amd/_build/libjfsx_FN1.so
JFSX_LIB=$F timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py tests/test_gpu_mirror.py tests/test_gpu_agg.py -q --timeout 120 --timeout-method thread > $out/t.log 2>&1
rc=$?; echo "FN1 tests rc $rc: $(tail -1 $out/t.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/t.log | head -5; exit 1; }
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --steps 5 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run main && JFSX_LIB=$F run fn1 && run main2 && JFSX_LIB=$F run fn1b && run open_main --mode open && JFSX_LIB=$F run open_fn1 --mode open || exit 1
for v in main FN1; do
  lib=juicefs_amd/_build/libjfsx_$v.so; [ $v = main ] && lib=juicefs_amd/libjfsx.so
  JFSX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 --steps 3 > $out/prof_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
  python3 - $out/prof_$v/run_kernel_stats.csv $v <<'PY'
import csv,sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'keysetup' in r['Name'] or 'finalize' in r['Name'] or 'main_k' in r['Name']: print(sys.argv[2], r['Name'][:28], round(float(r['AverageNs'])/1e3,1), 'us')
PY
done
