# Round-3 re-entry call 1: CRC byte-table parity + A/B, then the configs[1]-[4] bench lines.
set -u
cd "$GRAFT_REPO_ROOT"
bash scripts/gpu_r3_crcbyte.sh r3crc && bash scripts/gpu_r3_suite.sh r3s lines1
