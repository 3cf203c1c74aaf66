# Round-4 call 38: the AEAD kernels' block streams with non-temporal loads
# (ANT1) and loads + stores (ANT3) against the default: parity on each, then
# GCM seal (configs[1]) and ChaCha seal A/B, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4af; mkdir -p $out
export TMPDIR=/tmp
for v in ANT1 ANT3; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -q --timeout 120 --timeout-method thread > $out/t_$v.log 2>&1
  rc=$?; echo "$v tests rc $rc: $(tail -1 $out/t_$v.log)"; [ $rc -ne 0 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --steps 5 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); r=d['roofline']; print(sys.argv[2], 'value', d['value'], 'kernel_ms', r['kernel_avg_ms'])" $out/ab_$name.json $name; }
A1=juicefs_amd/_build/libjfsx_ANT1.so; A3=juicefs_amd/_build/libjfsx_ANT3.so
run gcm_base && JFSX_LIB=$A1 run gcm_nt1 && JFSX_LIB=$A3 run gcm_nt3 && run gcm_base2 && JFSX_LIB=$A1 run gcm_nt1b && JFSX_LIB=$A3 run gcm_nt3b && \
run cp_base --algo chacha20poly1305 && JFSX_LIB=$A3 run cp_nt3 --algo chacha20poly1305 && run cp_base2 --algo chacha20poly1305 && JFSX_LIB=$A3 run cp_nt3b --algo chacha20poly1305 && \
run crc_main --mode crc --steps 10
