# Round-4 call 2: unaligned-LDS probe; hybrid GCM kernel (BS = 2) parity, then
# a same-box A/B sweep of the hybrid split at 16 GiB (seal + CRC gen).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4b; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 60 ./tools/lds_unaligned > $out/lds_unaligned.txt 2>&1 || { echo "lds probe failed"; cat $out/lds_unaligned.txt; exit 1; }
cat $out/lds_unaligned.txt
JFSX_GCM_HYBRID=2,20,2 timeout -k 10 400 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fused_modes.py -x -q --timeout 120 --timeout-method thread > $out/hyb_pytest.log 2>&1 || { echo "hybrid parity failed"; tail -30 $out/hyb_pytest.log; exit 1; }
echo "hybrid parity: $(tail -1 $out/hyb_pytest.log)"
ab() {
  name=$1; shift
  env "$@" timeout -k 10 200 python3 bench.py --blocks 4096 --steps 5 --warmup 1 --no-cpu --verify 0 > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -5 $out/ab_$name.err; return 1; }
  python3 -c "import json; d=json.loads(open('$out/ab_$name.json').read().splitlines()[-1]); print('%-8s %s value %8.2f kernel_ms %7.3f' % ('$name', '$*', d['value'], d['roofline']['kernel_avg_ms']))"
}
ab base1 && ab h0 JFSX_GCM_HYBRID=0,16,0 && ab h1 JFSX_GCM_HYBRID=1,20,2 && \
ab h2r12 JFSX_GCM_HYBRID=2,12,2 && ab h2r20 JFSX_GCM_HYBRID=2,20,2 && ab h2r28 JFSX_GCM_HYBRID=2,28,2 && \
ab h2p0 JFSX_GCM_HYBRID=2,20,0 && ab h3 JFSX_GCM_HYBRID=3,20,2 && ab base2 || exit 1
# CRC-verify kernel variants (scripts/build_crc_variant.sh): byte tables with 2 / 4
# chains, quad-transposed coalesced loads (X) on the byte and nibble kernels
echo "crc A/B (64 GiB verify)"
AB_REPS="1 2" bash scripts/gpu_ab.sh r4crc "--mode crc" default=default b2=CRCB2 b4=CRCB4 bx2=CRCBX2 bx4=CRCBX4 nx=CRCNX
