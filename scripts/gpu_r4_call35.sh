# Round-4 call 35: RSA unwrap with a fixed 4-bit window (RWIN) against bit
# by bit (main): GPU RSA tests on RWIN, the zstd tests (5000-object round
# trip) on main, then the decrypt line (unwrap + open + verify) A/B, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ad; mkdir -p $out
export TMPDIR=/tmp
JFSX_LIB=juicefs_amd/_build/libjfsx_RWIN.so timeout -k 10 400 python3 -u -m pytest tests/test_gpu_rsa.py tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $out/t_rwin.log 2>&1
rc=$?; echo "RWIN tests rc $rc: $(tail -1 $out/t_rwin.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/t_rwin.log | head -5; exit 1; }
timeout -k 10 400 python3 -u -m pytest tests/test_gpu_zstdc.py tests/test_gpu_zstd.py -q --timeout 120 --timeout-method thread > $out/t.log 2>&1
rc=$?; echo "zstd tests rc $rc: $(tail -1 $out/t.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/t.log | head -5; exit 1; }
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --mode decrypt --steps 5 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run main && JFSX_LIB=juicefs_amd/_build/libjfsx_RWIN.so run rwin && run main2 && JFSX_LIB=juicefs_amd/_build/libjfsx_RWIN.so run rwin2
