# Round-4 call 3: GPU parity suite + smoke on the new CRC default; a same-box
# A/B of the 8-wave T-table shape with UR rows per iteration (JFSX_HYB_UR, env
# JFSX_GCM_HYBRID=0,16,0) against the 16-wave default; then one bench line per
# configs[1]-[4] mode with its same-run CPU baseline and the full oracle check
# of every block (scripts/gpu_r4_suite.sh lines1).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4c; mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_r3_tests.sh r4c || exit 1
JFSX_GCM_HYBRID=0,16,0 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -x -q --timeout 120 --timeout-method thread > $out/ur4_pytest.log 2>&1 || { echo "UR4 parity failed"; tail -30 $out/ur4_pytest.log; exit 1; }
echo "8-wave UR4 parity: $(tail -1 $out/ur4_pytest.log)"
JFSX_LIB=juicefs_amd/_build/libjfsx_HSWP4.so JFSX_GCM_HYBRID=0,16,0 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -x -q --timeout 120 --timeout-method thread > $out/swp_pytest.log 2>&1 || { echo "SWP parity failed"; tail -30 $out/swp_pytest.log; exit 1; }
echo "8-wave UR4 SWP parity: $(tail -1 $out/swp_pytest.log)"
ab() {
  name=$1; lib=$2; shift 2
  env JFSX_LIB=$lib "$@" timeout -k 10 200 python3 bench.py --blocks 4096 --steps 5 --warmup 1 --no-cpu --verify 0 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -5 $out/ab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/ab_$name.json').read().splitlines()[-1]); print('%-8s %s value %8.2f kernel_ms %7.3f' % ('$name', '$*', d['value'], d['roofline']['kernel_avg_ms']))"
}
D=juicefs_amd/libjfsx.so
ab base1 $D && ab ur4 $D JFSX_GCM_HYBRID=0,16,0 && ab ur3 juicefs_amd/_build/libjfsx_HUR3.so JFSX_GCM_HYBRID=0,16,0 && \
ab ur2 juicefs_amd/_build/libjfsx_HUR2.so JFSX_GCM_HYBRID=0,16,0 && ab ur4h2 $D JFSX_GCM_HYBRID=2,20,2 && \
ab ur4h1 $D JFSX_GCM_HYBRID=1,16,2 && ab swp4 juicefs_amd/_build/libjfsx_HSWP4.so JFSX_GCM_HYBRID=0,16,0 && \
ab base2 $D && ab ur4b $D JFSX_GCM_HYBRID=0,16,0 && ab swp4b juicefs_amd/_build/libjfsx_HSWP4.so JFSX_GCM_HYBRID=0,16,0 || exit 1
bash scripts/gpu_r4_suite.sh r4c lines1
