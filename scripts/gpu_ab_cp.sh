# Same-box A/B of ChaCha20-Poly1305 (full and ragged): default build vs _build/libjfsx_<variant>.so
# usage: bash scripts/gpu_ab_cp.sh <variant>
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/abcp
var=$1
for i in 1 2; do for v in default $var; do lib=juicefs_amd/libjfsx.so; [ $v = $var ] && lib=juicefs_amd/_build/libjfsx_$var.so
for m in "" "--ragged"; do
JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --algo chacha20poly1305 --no-cpu --verify 1 $m > gpurun_out/abcp/o.json 2>gpurun_out/abcp/o.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/abcp/o.json').read().strip().splitlines()[-1]); print('$v', '$m', d['value'], d['roofline']['kernel_avg_ms'])"; done; done; done
