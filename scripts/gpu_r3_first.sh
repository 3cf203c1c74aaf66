# Round-3 first contact: GPU tests, smoke and the default bench line on the
# round's starting tree.  usage: bash scripts/gpu_r3_first.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
bash scripts/gpu_full_tests.sh $1 || exit 1
timeout -k 10 420 python3 bench.py > $out/bench_seal_gcm.json 2> $out/bench_seal_gcm.err || { echo "bench failed"; tail -5 $out/bench_seal_gcm.err; exit 1; }
tail -1 $out/bench_seal_gcm.json | cut -c1-300
