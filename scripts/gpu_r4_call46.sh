# Round-4 call 46: with non-temporal loads, CRC verify with 4 interleaved
# span chains per lane (CH4) against the default 2: parity, then the 64 GiB
# crc line A/B, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ak; mkdir -p $out
export TMPDIR=/tmp
L=juicefs_amd/_build/libjfsx_CH4.so
JFSX_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -q --timeout 120 --timeout-method thread > $out/t.log 2>&1
rc=$?; echo "CH4 tests rc $rc: $(tail -1 $out/t.log)"; [ $rc -ne 0 ] && exit 1
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --mode crc --steps 10 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'value', d['value'], 'kernel_ms', r['kernel_avg_ms'], 'frac', r['frac'])" $out/ab_$name.json $name; }
run main && JFSX_LIB=$L run ch4 && run main2 && JFSX_LIB=$L run ch4b
