# Round-4 call 26: first-step width K0 = 1 for the zstd parser (default 2) and
# K0 = 2 / 1 for the LZ4 parser (default 4): parity, then 16 GiB text lines.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4z; mkdir -p $out
export TMPDIR=/tmp
for v in ZK1:tests/test_gpu_zstdc.py LK2:tests/test_gpu_lz4.py LK1:tests/test_gpu_lz4.py; do
  n=${v%%:*}; t=${v#*:}
  JFSX_LIB=juicefs_amd/_build/libjfsx_$n.so timeout -k 10 300 python3 -u -m pytest $t -q --timeout 120 --timeout-method thread > $out/t_$n.log 2>&1
  rc=$?; echo "$n rc $rc: $(tail -1 $out/t_$n.log)"; [ $rc -ne 0 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --blocks 4096 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run zbase --mode zstd --steps 2 --warmup 1 && JFSX_LIB=juicefs_amd/_build/libjfsx_ZK1.so run zk1 --mode zstd --steps 2 --warmup 1 && \
run lbase --mode lz4 && JFSX_LIB=juicefs_amd/_build/libjfsx_LK2.so run lk2 --mode lz4 && JFSX_LIB=juicefs_amd/_build/libjfsx_LK1.so run lk1 --mode lz4 && run lbase2 --mode lz4
