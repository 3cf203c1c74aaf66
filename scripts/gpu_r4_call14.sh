# Round-4 call 14: zstd compressor occupancy.  Work shrunk to 9.3 KiB (literal
# and sequence scratch in a union) and <= 128 VGPRs, so 16 waves per CU fit;
# parity of the default and the windowed parser (JFSX_ZC_WIN=3), then the
# 16 GiB text line per build x persistent waves per CU.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4n; mkdir -p $out
export TMPDIR=/tmp
for v in main Z3W; do
  lib=juicefs_amd/libjfsx.so; [ $v != main ] && lib=juicefs_amd/_build/libjfsx_$v.so
  JFSX_LIB=$lib timeout -k 10 200 python3 -u -m pytest tests/test_gpu_zstdc.py -q --timeout 120 --timeout-method thread > $out/t_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $out/t_$v.log)"
  [ $rc -ne 0 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 2 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run main_w8 && JFSX_ZC_WAVES=16 run main_w16 && \
JFSX_LIB=juicefs_amd/_build/libjfsx_Z3W.so JFSX_ZC_WAVES=8 run z3_w8 && \
JFSX_LIB=juicefs_amd/_build/libjfsx_Z3W.so JFSX_ZC_WAVES=16 run z3_w16 && \
JFSX_LIB=juicefs_amd/_build/libjfsx_Z3P3.so JFSX_ZC_WAVES=12 run z3p3_w12 && \
JFSX_LIB=juicefs_amd/_build/libjfsx_Z3W.so JFSX_ZC_WAVES=16 JFSX_ZC_QUEUE=1 run z3_w16q
