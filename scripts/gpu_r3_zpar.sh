# Block-parallel zstd decoder: GPU zstd tests, same-box A/B against the serial
# kernel (16 GiB of level-1 text), then the GPU suite, smoke and (optional) a
# section of the r3 measurement suite.  usage: bash scripts/gpu_r3_zpar.sh <tag> [section]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_zstd.py > $out/pytest_zstd.log 2>&1 || { echo "zstd tests failed"; tail -40 $out/pytest_zstd.log; exit 1; }
echo "zstd tests: $(tail -1 $out/pytest_zstd.log)"
for rep in 1; do
  JFSX_ZSTD_SERIAL=1 timeout -k 10 300 python3 bench.py --mode unzstd --blocks 4096 --no-cpu --steps 3 --warmup 1 > $out/unzstd_serial.$rep.json 2> $out/unzstd_serial.$rep.err || { echo "serial bench failed"; tail -5 $out/unzstd_serial.$rep.err; exit 1; }
  timeout -k 10 300 python3 bench.py --mode unzstd --blocks 4096 --no-cpu --steps 5 --warmup 1 > $out/unzstd_par.$rep.json 2> $out/unzstd_par.$rep.err || { echo "par bench failed"; tail -5 $out/unzstd_par.$rep.err; exit 1; }
  for v in serial par; do echo "unzstd $v.$rep: $(python3 -c "import json; d=json.loads(open('$out/unzstd_$v.$rep.json').read().splitlines()[-1]); print(d['value'], d['roofline']['kernel_avg_ms'], d['roofline'].get('objects_to_serial_decoder'))")"; done
done
if [ -n "${ZSTAMP:-}" ]; then
  JFSX_LIB=juicefs_amd/_build/libjfsx_$ZSTAMP.so timeout -k 10 200 python3 scripts/zstd_stamps.py 512 > $out/stamps_par.txt 2>&1 || { echo "stamps failed"; tail -20 $out/stamps_par.txt; exit 1; }
  cat $out/stamps_par.txt
fi
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest.log 2>&1 || { echo "gpu tests failed"; tail -30 $out/pytest.log; exit 1; }
echo "gpu tests: $(tail -1 $out/pytest.log)"
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $out/smoke.log; exit 1; }
echo "smoke: $(tail -1 $out/smoke.log)"
if [ $# -ge 2 ]; then bash scripts/gpu_r3_suite.sh $1 $2; fi
