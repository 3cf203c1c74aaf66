# zstd block-parallel decoder: GPU zstd tests, stamps of the ZSTAMP2 build,
# one same-box A/B pair.  usage: bash scripts/gpu_r3_zst2.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_zstd.py > $out/pytest_zstd.log 2>&1 || { echo "zstd tests failed"; tail -40 $out/pytest_zstd.log; exit 1; }
echo "zstd tests: $(tail -1 $out/pytest_zstd.log)"
JFSX_LIB=juicefs_amd/_build/libjfsx_ZSTAMP2.so timeout -k 10 200 python3 scripts/zstd_stamps.py 512 > $out/stamps_par.txt 2>&1 || { echo "stamps failed"; tail -20 $out/stamps_par.txt; exit 1; }
cat $out/stamps_par.txt
timeout -k 10 300 python3 bench.py --mode unzstd --blocks 4096 --no-cpu --steps 5 --warmup 1 > $out/unzstd_par.json 2> $out/unzstd_par.err || { echo "par bench failed"; tail -5 $out/unzstd_par.err; exit 1; }
echo "unzstd par: $(python3 -c "import json; d=json.loads(open('$out/unzstd_par.json').read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'], d['roofline'].get('objects_to_serial_decoder'))")"
