# Round-4 call 37: CRC verify with non-temporal loads (CNT) against the
# default: parity on CNT, then the 64 GiB crc line A/B, two reps each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ae; mkdir -p $out
export TMPDIR=/tmp
JFSX_LIB=juicefs_amd/_build/libjfsx_CNT.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -q --timeout 120 --timeout-method thread > $out/t_cnt.log 2>&1
rc=$?; echo "CNT tests rc $rc: $(tail -1 $out/t_cnt.log)"; [ $rc -ne 0 ] && exit 1
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --mode crc --steps 10 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'value', d['value'], 'kernel_ms', r['kernel_avg_ms'], 'frac', r['frac'])" $out/ab_$name.json $name; }
run base && JFSX_LIB=juicefs_amd/_build/libjfsx_CNT.so run nt && run base2 && JFSX_LIB=juicefs_amd/_build/libjfsx_CNT.so run nt2
