# Round-4 call 28: zstd compressor entropy-stage loops and block copies with several loads in flight (JFSX_ZC_MLP=1, main) against the one-load-per-iteration loops (ZM0)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4mlp; mkdir -p $out
export TMPDIR=/tmp
vs="${VS:-ZM0 ZM1 ZM30}"
for v in main $vs; do
  lib=juicefs_amd/_build/libjfsx_$v.so; [ $v = main ] && lib=juicefs_amd/libjfsx.so
  JFSX_LIB=$lib timeout -k 10 200 python3 -u -m pytest tests/test_gpu_zstdc.py -q --timeout 120 --timeout-method thread > $out/t_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $out/t_$v.log)"
  [ $rc -ne 0 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 2 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run base || exit 1
for v in $vs; do JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so run $v || exit 1; done
run base2
run rbase --lz4-data random && JFSX_LIB=juicefs_amd/_build/libjfsx_ZM0.so run rzm0 --lz4-data random && JFSX_LIB=juicefs_amd/_build/libjfsx_ZM1.so run rzm1 --lz4-data random
