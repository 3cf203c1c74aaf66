# Round-4 call 13: the register-window zstd parser after the masked-lane
# ds_bpermute fix (repcode check), byte-for-byte test per JFSX_ZC_WIN variant,
# then the 16 GiB text line for each passing variant against the default.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4m; mkdir -p $out
export TMPDIR=/tmp
pass=""
for v in 1 3 17 31; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_ZW$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_zstdc.py -q --timeout 120 --timeout-method thread > $out/zw${v}.log 2>&1
  rc=$?
  echo "ZW$v rc $rc: $(tail -1 $out/zw${v}.log)"
  grep -o "At index [0-9]* diff" $out/zw${v}.log | head -3
  if [ $rc -eq 0 ]; then pass="$pass $v"; fi
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; exit 1; fi
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 3 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'])" $out/ab_$name.json $name; }
run base || exit 1
for v in $pass; do JFSX_LIB=juicefs_amd/_build/libjfsx_ZW$v.so run zw$v || exit 1; done
run base2
