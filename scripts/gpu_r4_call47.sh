# Round-4 call 47: the launcher path the driver uses for its SCALE runs, at
# one rank on this one-GPU box: torch.distributed.run -> bench.py (RCCL
# barrier and max-over-ranks timing), default workload.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4al; mkdir -p $out
export TMPDIR=/tmp
timeout -k 10 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --steps 5 --warmup 1 > $out/dist1.json 2> $out/dist1.err
rc=$?; echo "rc $rc"; tail -1 $out/dist1.json | cut -c1-300; [ $rc -ne 0 ] && tail -20 $out/dist1.err
exit $rc
