# Round-4 call 5: codec and per-object lines with their same-run CPU baselines
# (scripts/gpu_r4_suite.sh lines2): LZ4 / zstd compress and decompress of 16 GiB
# of text, the block-parallel zstd decoder at 64 GiB, the aggregator at 20 and
# 32 threads, the four codec directions through the aggregator.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r4_suite.sh r4e lines2
# host ingest again with the PCIe probe on ring-like buffers, before and after the ring
out=gpurun_out/suite_r4e
timeout -k 10 500 python3 bench.py --mem host --blocks 2048 --steps 8 --warmup 1 > $out/bench_ingest_gcm.json 2> $out/bench_ingest_gcm.err || { echo "ingest failed"; tail -5 $out/bench_ingest_gcm.err; exit 1; }
echo "ingest: $(tail -1 $out/bench_ingest_gcm.json | cut -c1-200)"
