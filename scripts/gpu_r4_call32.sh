# Round-4 call 32: SQ passes (LDS / VALU busy) for the lines that had none:
# ChaCha open, the ragged configs[4] lines, and LZ4 decompression.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_r4h2; mkdir -p $out
export TMPDIR=/tmp
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQ="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
SQC="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
pmc open_chacha__sq "$SQ" --blocks 1024 --mode open --algo chacha20poly1305 && \
pmc seal_gcm_ragged__sq "$SQ" --ragged && pmc open_gcm_ragged__sq "$SQ" --ragged --mode open && \
pmc seal_chacha_ragged__sq "$SQ" --ragged --algo chacha20poly1305 && pmc open_chacha_ragged__sq "$SQ" --ragged --mode open --algo chacha20poly1305 && \
pmc unlz4_text__sq "$SQC" --mode unlz4 --blocks 4096
