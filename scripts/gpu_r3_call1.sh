# Round-3 re-entry call (short): CRC byte-table parity + A/B, then the headline
# seal line and the CRC-verify line with their same-run CPU baselines.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_r3s; mkdir -p $out
bash scripts/gpu_r3_crcbyte.sh r3crc && \
timeout -k 10 300 python3 bench.py > $out/bench_seal_gcm.json 2> $out/bench_seal_gcm.err && echo "seal: $(tail -1 $out/bench_seal_gcm.json | cut -c1-200)" && \
timeout -k 10 300 python3 bench.py --mode crc > $out/bench_crc_verify.json 2> $out/bench_crc_verify.err && echo "crc: $(tail -1 $out/bench_crc_verify.json | cut -c1-200)"
