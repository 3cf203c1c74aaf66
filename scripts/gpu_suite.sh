# Full measurement suite for one round: benches for every config + rocprof stats.
# usage: bash scripts/gpu_suite.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
tag=$1
out=gpurun_out/suite_$tag
mkdir -p $out
export TMPDIR=/tmp
run() { name=$1; shift; timeout -k 10 600 python3 bench.py "$@" > $out/$name.json 2> $out/$name.err || { echo "$name failed"; tail -5 $out/$name.err; return 1; }; echo "$name: $(tail -1 $out/$name.json | cut -c1-160)"; }
run seal_gcm && \
run seal_chacha --algo chacha20poly1305 --no-cpu && \
run open_gcm --mode open --no-cpu && \
run open_chacha --mode open --algo chacha20poly1305 --no-cpu && \
run crc_verify --mode crc --no-cpu && \
run ingest_gcm --mem host --blocks 2048 --steps 16 --warmup 1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof -o run --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu --verify 0 > $out/prof.log 2>&1 && \
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $out/prof_cp -o run --output-format csv -- python3 bench.py --algo chacha20poly1305 --steps 3 --warmup 1 --no-cpu --verify 0 > $out/prof_cp.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d $out/pmc1 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 > $out/pmc1.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --pmc WRITE_SIZE -d $out/pmc2 -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 > $out/pmc2.log 2>&1 && \
python3 scripts/pmc_summary.py $out > $out/pmc_summary.txt && echo suite done
