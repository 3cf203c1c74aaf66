# JFSX_AGG_INFLIGHT 2 / 3 / 4 on the current build (keysetup stream, 21 us keysetup), heap Encrypt, no CPU leg
set -u
t=${1:-r6i3}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --no-cpu --warmup-seconds 3"
for sz in 65536:400 262144:100 1048576:30; do
  b=${sz%%:*}; n=${sz##*:}
  for f in 2 3 4; do JFSX_AGG_INFLIGHT=$f $S if${f}_$b $A --block-bytes $b --steps $n || exit 1; done
done
for f in 2 3; do JFSX_AGG_INFLIGHT=$f $S if${f}_ragged $A --ragged --steps 20 || exit 1; done
