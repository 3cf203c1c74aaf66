# Zstandard decompression: GPU parity tests, then 16 GiB bench lines (text /
# random).  usage: bash scripts/gpu_zstd.sh <tag> [blocks]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/zstd_$1
mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests/test_gpu_zstd.py -x -q -m gpu --timeout 300 --timeout-method thread > $out/pytest.log 2>&1
rc=$?
tail -2 $out/pytest.log
[ $rc -eq 0 ] || { grep -E 'FAIL|Error|assert' $out/pytest.log | head -20; exit 1; }
for d in text random; do
  timeout -k 10 400 python3 bench.py --mode unzstd --lz4-data $d --blocks ${2:-4096} --steps 2 --warmup 1 ${NOCPU:-} > $out/unzstd_$d.json 2> $out/unzstd_$d.err || { tail -5 $out/unzstd_$d.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$out/unzstd_$d.json').read().strip().splitlines()[-1]); print('$d', d['value'], d['roofline']['kernel_avg_ms'], d['config']['ratio'], d['cpu_baseline'] and d['cpu_baseline']['value'])"
done
