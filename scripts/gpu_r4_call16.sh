# Round-4 call 16: zstd compressor at 16 waves per CU -- the windowed parser
# with everything after a match from windows (JFSX_ZC_WIN=31) at K0 = 2 / 3,
# and FETCH_SIZE per launch for 3 / 31 / 35 / 99 (is the parser fetch-bound?)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4p; mkdir -p $out
export TMPDIR=/tmp JFSX_ZC_WAVES=16
for v in ZW31K2 ZW31K3; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so timeout -k 10 200 python3 -u -m pytest tests/test_gpu_zstdc.py -q --timeout 120 --timeout-method thread > $out/t_$v.log 2>&1
  rc=$?; echo "$v rc $rc: $(tail -1 $out/t_$v.log)"
  [ $rc -gt 1 ] && exit 1
done
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 2 --warmup 1 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
for v in ZW31 ZW31K2 ZW31K3; do JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so run $v || exit 1; done
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 --mode zstd --blocks 4096 > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; python3 - $out/pmc_$name <<'PY'
import csv,glob,sys
for f in glob.glob(sys.argv[1]+'/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'zstd_compress' in r.get('Kernel_Name',''): print(sys.argv[1].split('/')[-1], r['Counter_Name'], r['Counter_Value'])
PY
}
for v in Z3W ZW31 ZW35 ZW99; do JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so pmc f_$v FETCH_SIZE || exit 1; done
