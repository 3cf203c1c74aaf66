# Round-4 call 31: GCM keysetup with its T0 / T2 lookups from an LDS copy
# (main) against the global-table build (KOLD): parity, then the configs[1]
# step and the keysetup kernel's rocprof time for each, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ab; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -q --timeout 120 --timeout-method thread > $out/t_main.log 2>&1
rc=$?; echo "main rc $rc: $(tail -1 $out/t_main.log)"; [ $rc -ne 0 ] && exit 1
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --steps 5 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run main && JFSX_LIB=juicefs_amd/_build/libjfsx_KOLD.so run old && run main2 && JFSX_LIB=juicefs_amd/_build/libjfsx_KOLD.so run old2 || exit 1
for v in main KOLD; do
  lib=juicefs_amd/_build/libjfsx_$v.so; [ $v = main ] && lib=juicefs_amd/libjfsx.so
  JFSX_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $out/prof_$v -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 --steps 3 > $out/prof_$v.log 2>&1 || { echo "prof $v failed"; exit 1; }
  grep -h "keysetup\|finalize" $out/prof_$v/run_kernel_stats.csv | cut -d, -f1,4 | sed "s/^/$v /" | cut -c1-160
done
