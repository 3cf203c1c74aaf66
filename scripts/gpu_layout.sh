# ragged GCM: is it the size mix or the 4 MiB-slot layout?
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/layout
mkdir -p $out
run() { name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 1 --steps 5 "$@" > $out/$name.log 2>&1 || { echo "$name failed"; tail -3 $out/$name.log; return 1; }
  python3 -c "import json; d=json.loads(open('$out/$name.log').read().strip().splitlines()[-1]); print('%-16s %8.1f GB/s  kernel %.3f ms' % ('$name', d['value'], d['roofline']['kernel_avg_ms']))"; }
run fix2M_dense --blocks 4096 --block-bytes 2097152 && run fix2M_slot4M --blocks 4096 --fixed-len 2097152 && \
run rag_slot4M --blocks 4096 --ragged && run rag_packed --blocks 4096 --ragged --packed && \
run fix2M_dense_b --blocks 4096 --block-bytes 2097152 && run rag_slot4M_b --blocks 4096 --ragged
