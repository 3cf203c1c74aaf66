set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
export TMPDIR=/tmp
rocminfo 2>/dev/null | grep -m3 -E "gfx|Marketing" > gpurun_out/r1_info.log || true
nproc >> gpurun_out/r1_info.log
timeout -k 10 420 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/r1_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc"
tail -30 gpurun_out/r1_pytest.log
if [ $rc -le 1 ]; then
  timeout -k 10 300 python bench.py --blocks 1024 --steps 5 --warmup 1 --no-cpu > gpurun_out/r1_bench_small.log 2>&1
  echo "bench rc=$?"
  cat gpurun_out/r1_bench_small.log | tail -5
fi
