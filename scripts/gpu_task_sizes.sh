# GCM seal+CRC kernel time per byte against block size and raggedness (8 GiB-ish batches)
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/tsize
mkdir -p $out
run() { name=$1; shift; timeout -k 10 200 python3 bench.py --no-cpu --verify 1 --steps 5 "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.log; return 1; }
  python3 -c "import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('%-14s %8.1f GB/s  kernel %.3f ms' % ('$name', d['value'], d['roofline']['kernel_avg_ms']))"; }
run fix4M --blocks 2048 && run fix2M --blocks 4096 --block-bytes 2097152 && run fix1M --blocks 8192 --block-bytes 1048576 && \
run fix256K --blocks 32768 --block-bytes 262144 && run fix64K --blocks 131072 --block-bytes 65536 && \
run rag --blocks 4096 --ragged && run rag_a32K --blocks 4096 --ragged --ragged-align 32768 && run rag_a1K --blocks 4096 --ragged --ragged-align 1024 && run rag_a2K --blocks 4096 --ragged --ragged-align 2048
