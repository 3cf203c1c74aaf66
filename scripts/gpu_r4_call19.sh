# Round-4 call 19: zstd parser variants (VS; 159 = 31 + 128 repcode windows, 287 = 31 + 256 candidate extensions)
# against the default (31): parity, then the 16 GiB text line, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4s; mkdir -p $out
export TMPDIR=/tmp
vs="${VS:-ZW287 ZW415}"
for v in $vs; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_zstdc.py -q --timeout 120 --timeout-method thread > $out/t_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $out/t_$v.log)"
  [ $rc -ne 0 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 2 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run base || exit 1
for v in $vs; do JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so run $v || exit 1; done
run base2
