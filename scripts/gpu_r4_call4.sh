# Round-4 call 4: PMC passes the bench lines read (scripts/pmc_r3.py):
# FETCH / WRITE of the second half of the configs and the codecs, the CRC-verify
# kernel again (new default), SQ busy counters of CRC verify and the codecs,
# then rocprofv3 kernel stats at the bench lines' own sizes.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_r4d; mkdir -p $out
export TMPDIR=/tmp
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQ="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
SQC="SQ_INSTS_SALU SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE"
Z="--blocks 4096"
pmc crc_verify__fetch FETCH_SIZE --mode crc && pmc crc_verify__write WRITE_SIZE --mode crc && \
pmc crc_verify__sq "$SQ" --blocks 1024 --mode crc && \
pmc seal_chacha_ragged__fetch FETCH_SIZE --ragged --algo chacha20poly1305 && pmc seal_chacha_ragged__write WRITE_SIZE --ragged --algo chacha20poly1305 && \
pmc open_chacha_ragged__fetch FETCH_SIZE --ragged --mode open --algo chacha20poly1305 && pmc open_chacha_ragged__write WRITE_SIZE --ragged --mode open --algo chacha20poly1305 && \
pmc ingest_gcm__fetch FETCH_SIZE --mem host --blocks 2048 && pmc ingest_gcm__write WRITE_SIZE --mem host --blocks 2048 && \
pmc zstd_text__fetch FETCH_SIZE --mode zstd $Z && pmc zstd_text__write WRITE_SIZE --mode zstd $Z && pmc zstd_text__sq "$SQC" --mode zstd --blocks 1024 && \
pmc unzstd_text__fetch FETCH_SIZE --mode unzstd $Z && pmc unzstd_text__write WRITE_SIZE --mode unzstd $Z && pmc unzstd_text__sq "$SQC" --mode unzstd --blocks 1024 && \
pmc lz4_text__fetch FETCH_SIZE --mode lz4 $Z && pmc lz4_text__write WRITE_SIZE --mode lz4 $Z && \
pmc unlz4_text__fetch FETCH_SIZE --mode unlz4 $Z && pmc unlz4_text__write WRITE_SIZE --mode unlz4 $Z || exit 1
bash scripts/gpu_r4_suite.sh r4d prof
