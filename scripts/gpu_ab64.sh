# Same-box A/B at the full 64 GiB bench size: default build vs juicefs_amd/_build/libjfsx_<variant>.so
# usage: bash scripts/gpu_ab64.sh <variant>
set -u
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out/ab
var=$1
for i in 1 2; do for v in default $var; do lib=juicefs_amd/libjfsx.so; [ $v = $var ] && lib=juicefs_amd/_build/libjfsx_$var.so
JFSX_LIB=$lib timeout -k 10 300 python3 bench.py --no-cpu --verify 1 > gpurun_out/ab/$v$i.json 2>gpurun_out/ab/$v$i.err || exit 1
python3 -c "import json; d=json.loads(open('gpurun_out/ab/$v$i.json').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"; done; done
