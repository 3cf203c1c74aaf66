# Round-4 call 30: LZ4 compressor literal copy from the window looping only
# over the 64-byte groups the run needs (main) against the 4-group loop (LOLD).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4aa; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lz4.py -q --timeout 120 --timeout-method thread > $out/t_main.log 2>&1
rc=$?; echo "main rc $rc: $(tail -1 $out/t_main.log)"; [ $rc -ne 0 ] && exit 1
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --blocks 4096 --mode lz4 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run main && JFSX_LIB=juicefs_amd/_build/libjfsx_LOLD.so run old && run main2 && JFSX_LIB=juicefs_amd/_build/libjfsx_LOLD.so run old2
