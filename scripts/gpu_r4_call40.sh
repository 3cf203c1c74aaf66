# Round-4 call 40: the remaining GCM-kernel lines on the final build (bitsliced
# AES seal, decrypt, host ingest) with same-run CPU baselines and full checks.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_r4k2; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 700 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-110)"; }
run seal_gcm_bitslice --aes bitslice && run decrypt_gcm --mode decrypt && run ingest_gcm --mem host --steps 8 --warmup 1
