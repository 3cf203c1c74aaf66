# Round-4 call 15: at 16 waves per CU, the windowed parser's feature bits
# (JFSX_ZC_WIN 3 / 19 / 31 / 35 / 99) and the speculation width K0 (2 / 4 / 8),
# 16 GiB of text; parity of each build first.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4o; mkdir -p $out
export TMPDIR=/tmp JFSX_ZC_WAVES=16
vs="Z3W ZW35 ZW99 ZW19 ZW31 Z3K2 Z3K8"
for v in $vs; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_zstdc.py -q --timeout 120 --timeout-method thread > $out/t_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $out/t_$v.log)"
  [ $rc -gt 1 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 2 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
for v in $vs Z3W; do JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so run $v || exit 1; done
