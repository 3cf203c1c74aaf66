# Round-4 call 33: the codec compress lines on the final build -- LZ4 text
# (16 GiB) and zstd text at 64 GiB -- with their same-run CPU baselines, and
# the LZ4 compressor's rocprof stats.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_r4i2; mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-150)"; }
timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_lz4_text -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 --mode lz4 --blocks 4096 --steps 3 --warmup 1 > $out/prof_lz4_text.log 2>&1 && echo "prof lz4 ok" || exit 1
run lz4_text --mode lz4 --blocks 4096 && run zstd_text_64g --mode zstd --blocks 16384 --steps 2 --warmup 1
