# Round-4 call 21: host-trap PC sampling of the zstd compressor (where the
# parse's instructions and stalls are), 1024 objects.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4u; mkdir -p $out
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method host_trap --pc-sampling-unit time --pc-sampling-interval 100 -d $out/pcs -o run --output-format csv -- python3 bench.py --mode zstd --blocks 1024 --steps 1 --warmup 0 --no-cpu --verify 0 > $out/pcs.log 2>&1
rc=$?; echo "rc $rc"; grep -v "^ *@" $out/pcs.log | tail -5; ls -la $out/pcs/* 2>/dev/null | head; find $out/pcs -name "*.csv" | head
