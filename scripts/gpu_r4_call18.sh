# Round-4 call 18: zstd compressor section stamps on the new defaults (parse vs
# entropy ticks per object), then the codec compress lines on random data and
# the zstd text line at 64 GiB, each with its same-run CPU baseline.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4r; mkdir -p $out
export TMPDIR=/tmp
JFSX_LIB=juicefs_amd/_build/libjfsx_ZSTAMP.so timeout -k 10 200 python3 bench.py --no-cpu --verify 0 --mode zstd --blocks 4096 --steps 1 --warmup 0 > $out/stamp.log 2>&1 || { echo "stamp failed"; tail -5 $out/stamp.log; exit 1; }
grep "zc-stamp" $out/stamp.log | head -4
run() { local name=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-200)"; }
run zstd_random --mode zstd --lz4-data random --blocks 4096 --steps 3 --warmup 1 && \
run lz4_random --mode lz4 --lz4-data random --blocks 4096 && \
run zstd_text_64g --mode zstd --blocks 16384 --steps 2 --warmup 1
