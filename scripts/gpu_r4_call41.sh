# Round-4 call 41: the ChaCha kernel with non-temporal loads only (CPNT1;
# its stores keep the default policy) against the default, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4ag; mkdir -p $out
export TMPDIR=/tmp
JFSX_LIB=juicefs_amd/_build/libjfsx_CPNT1.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -q --timeout 120 --timeout-method thread > $out/t.log 2>&1
rc=$?; echo "CPNT1 tests rc $rc: $(tail -1 $out/t.log)"; [ $rc -ne 0 ] && exit 1
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --steps 5 --algo chacha20poly1305 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'value', d['value'], 'kernel_ms', r['kernel_avg_ms'])" $out/ab_$name.json $name; }
L=juicefs_amd/_build/libjfsx_CPNT1.so
run base && JFSX_LIB=$L run nt1 && run base2 && JFSX_LIB=$L run nt1b
