# Measurement suite (rounds 3-4): one bench line per BASELINE config and mode, each
# with its same-run CPU baseline; rocprofv3 kernel stats at the bench lines'
# own configs; PMC passes named pmc_<variant>__<set> for scripts/pmc_r3.py
# (FETCH/WRITE at the bench size, SQ busy counters on a 4 GiB batch).
# usage: bash scripts/gpu_r4_suite.sh <tag> [lines1|lines2|prof|pmc1|pmc1a|pmc1b|pmc2|all]
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/suite_$1
what=${2:-all}
mkdir -p $out
export TMPDIR=/tmp
run() { local name=$1; shift; timeout -k 10 500 python3 bench.py "$@" > $out/bench_$name.json 2> $out/bench_$name.err || { echo "$name failed"; tail -5 $out/bench_$name.err; return 1; }; echo "$name: $(tail -1 $out/bench_$name.json | cut -c1-160)"; }
prof() { local name=$1; shift; timeout -k 10 500 rocprofv3 --kernel-trace --stats -d $out/prof_$name -o run --output-format csv -- python3 bench.py --no-cpu --verify 0 "$@" > $out/prof_$name.log 2>&1 || { echo "prof $name failed"; tail -5 $out/prof_$name.log; return 1; }; echo "prof $name ok"; }
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; echo "pmc $name ok"; }
SQ="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
Z="--blocks 4096"   # codec lines: 16 GiB
if [ $what = lines1 ] || [ $what = all ]; then
run seal_gcm && \
run seal_gcm_bitslice --aes bitslice && \
run seal_chacha --algo chacha20poly1305 && \
run open_gcm --mode open && \
run open_chacha --mode open --algo chacha20poly1305 && \
run crc_verify --mode crc && \
run seal_gcm_ragged --ragged && run open_gcm_ragged --ragged --mode open && \
run seal_chacha_ragged --ragged --algo chacha20poly1305 && run open_chacha_ragged --ragged --mode open --algo chacha20poly1305 && \
run decrypt_gcm --mode decrypt && \
run ingest_gcm --mem host --blocks 2048 --steps 8 --warmup 1 || exit 1
fi
if [ $what = lines2 ] || [ $what = all ]; then
run lz4_text --mode lz4 $Z && run unlz4_text --mode unlz4 $Z && \
run zstd_text --mode zstd $Z --steps 3 --warmup 1 && run unzstd_text --mode unzstd $Z && \
run agg_gcm_t20 --mode agg --threads 20 --steps 5 --warmup 1 && run agg_gcm_t32 --mode agg --threads 32 --steps 5 --warmup 1 && \
run aggcodec_lz4 --mode aggcodec --codec lz4 --threads 20 --steps 2 --warmup 1 && \
run aggcodec_unlz4 --mode aggcodec --codec unlz4 --threads 20 --steps 2 --warmup 1 && \
run aggcodec_zstd --mode aggcodec --codec zstd --threads 20 --steps 2 --warmup 1 && \
run aggcodec_unzstd --mode aggcodec --codec unzstd --threads 20 --steps 2 --warmup 1 && \
run unzstd_text_64g --mode unzstd --steps 5 --warmup 1 || exit 1
fi
if [ $what = agg_codec_zstd ]; then
run aggcodec_zstd --mode aggcodec --codec zstd --threads 20 --steps 2 --warmup 1 && \
run aggcodec_unzstd --mode aggcodec --codec unzstd --threads 20 --steps 2 --warmup 1 || exit 1
fi
if [ $what = prof ] || [ $what = all ]; then
prof gcm --steps 10 --warmup 2 && prof gcm_ragged --ragged --steps 10 --warmup 2 && \
prof open_gcm --mode open --steps 10 --warmup 2 && \
prof cp --algo chacha20poly1305 --steps 10 --warmup 2 && prof crc --mode crc --steps 10 --warmup 2 && \
prof zstd_text --mode zstd $Z --steps 3 --warmup 1 && prof unzstd_text --mode unzstd $Z --steps 10 --warmup 2 && \
prof lz4_text --mode lz4 $Z --steps 10 --warmup 2 && prof unlz4_text --mode unlz4 $Z --steps 10 --warmup 2 || exit 1
fi
P1A='"seal_gcm:" "open_gcm:--mode open" "seal_chacha:--algo chacha20poly1305" "open_chacha:--mode open --algo chacha20poly1305" "crc_verify:--mode crc" "seal_gcm_ragged:--ragged" "open_gcm_ragged:--ragged --mode open"'
P1B='"seal_chacha_ragged:--ragged --algo chacha20poly1305" "open_chacha_ragged:--ragged --mode open --algo chacha20poly1305" "ingest_gcm:--mem host --blocks 2048" "zstd_text:--mode zstd $Z" "unzstd_text:--mode unzstd $Z" "lz4_text:--mode lz4 $Z" "unlz4_text:--mode unlz4 $Z"'
case $what in pmc1) P1="$P1A $P1B";; pmc1a) P1=$P1A;; pmc1b) P1=$P1B;; all) P1="$P1A $P1B";; *) P1="";; esac
eval "set -- $P1"
for v in "$@"; do
  name=${v%%:*}; a=${v#*:}
  pmc ${name}__fetch FETCH_SIZE $a && pmc ${name}__write WRITE_SIZE $a || exit 1
done
if [ $what = pmc2 ] || [ $what = all ]; then
for v in "seal_gcm:" "open_gcm:--mode open" "seal_chacha:--algo chacha20poly1305" "crc_verify:--mode crc" \
         "seal_gcm_bitslice:--aes bitslice"; do
  name=${v%%:*}; a=${v#*:}
  pmc ${name}__sq "$SQ" --blocks 1024 $a || exit 1
done
echo "pmc2 done (summary: python3 scripts/pmc_r3.py gpurun_out/suite_<tag> on the merged passes)"
fi
