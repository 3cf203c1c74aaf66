set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
for v in gh8 u2; do
 for c in full none; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_$v.so timeout -k 10 120 python3 bench.py --blocks 2048 --steps 5 --warmup 1 --no-cpu --verify 0 --crc $c > gpurun_out/cs_${v}_$c.log 2>&1 || { tail -3 gpurun_out/cs_${v}_$c.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cs_${v}_$c.log').read().strip().splitlines()[-1]); print('$v $c', d['value'], d['roofline']['kernel_avg_ms'])"
 done
done
