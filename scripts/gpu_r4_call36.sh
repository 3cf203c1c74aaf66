# Round-4 call 36: what the round-end driver runs on the current tree
# (pytest -m gpu, smoke(), bench.py with no flags), plus the decrypt line
# (RSA unwrap + Open + verify) with its same-run CPU baseline.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_tests.sh r4f3 || exit 1
out=gpurun_out/r4f3; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 bench.py > $out/bench_default.json 2> $out/bench_default.err || { echo "bench failed"; tail -5 $out/bench_default.err; exit 1; }
echo "bench: $(tail -1 $out/bench_default.json | cut -c1-160)"
timeout -k 10 600 python3 bench.py --mode decrypt > $out/bench_decrypt_gcm.json 2> $out/bench_decrypt_gcm.err || { echo "decrypt failed"; tail -5 $out/bench_decrypt_gcm.err; exit 1; }
echo "decrypt: $(tail -1 $out/bench_decrypt_gcm.json | cut -c1-160)"
