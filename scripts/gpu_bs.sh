# Bitsliced-AES GCM variants: timing (8 GiB seal) + one PMC pass on the default build.
set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bs
export TMPDIR=/tmp
B="python3 bench.py --blocks 2048 --steps 5 --warmup 1 --no-cpu --verify 1"
run() { v=$1; lib=$2; shift 2; JFSX_LIB=$lib timeout -k 10 120 $B "$@" > gpurun_out/bs/$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/bs/$v.log; return 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/bs/$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"; }
for spec in "$@"; do
  v=${spec%%:*}; rest=${spec#*:}; lib=${rest%%:*}; args=""; [ "$rest" != "$lib" ] && args=${rest#*:}
  run $v $lib $args || exit 1
done
