# Full measurement suite for one round: benches for every config + rocprof stats + PMC traffic.
# usage: bash scripts/gpu_suite.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1
out=gpurun_out/suite_$tag
mkdir -p $out
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -5 $out/$name.err; return 1; }; echo "$name: $(tail -1 $out/$name.json | cut -c1-160)"; }
prof() { name=$1; shift; timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/$name -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --verify 0 "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }; }
pmc() { name=$1; ctr=$2; shift 2; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -5 $out/$name.log; return 1; }; }
run seal_gcm && \
run seal_gcm_bitslice --aes bitslice --no-cpu && \
run seal_chacha --algo chacha20poly1305 --no-cpu && \
run open_gcm --mode open --no-cpu && \
run open_chacha --mode open --algo chacha20poly1305 --no-cpu && \
run crc_verify --mode crc --no-cpu && \
run ingest_gcm --mem host --blocks 2048 --steps 8 --warmup 1 --no-cpu && \
prof prof_gcm && prof prof_gcm_bs --aes bitslice && prof prof_cp --algo chacha20poly1305 && prof prof_crc --mode crc && \
pmc pmc_gcm_fetch FETCH_SIZE && pmc pmc_gcm_write WRITE_SIZE && \
pmc pmc_cp_fetch FETCH_SIZE --algo chacha20poly1305 && pmc pmc_cp_write WRITE_SIZE --algo chacha20poly1305 && \
pmc pmc_crc_fetch FETCH_SIZE --mode crc && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo suite done
