# A/B of the host pipeline's keysetup stream (JFSX_KS_STREAM=1 default vs 0)
# on per-object heap Encrypt / Decrypt by block size (no CPU leg), after the GPU tests.
set -u
t=${1:-r6w}
S="bash scripts/suite.sh $t"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3"
$S tests || exit 1
for sz in 65536:400 262144:100 1048576:30 4194304:10; do
  b=${sz%%:*}; n=${sz##*:}
  $S line ks1_$b $A --agg-op seal --block-bytes $b --steps $n || exit 1
  JFSX_KS_STREAM=0 $S line ks0_$b $A --agg-op seal --block-bytes $b --steps $n || exit 1
done
$S line ks1_open $A --agg-op open --steps 10 || exit 1
JFSX_KS_STREAM=0 $S line ks0_open $A --agg-op open --steps 10 || exit 1
$S line ks1_ingest --mem host --steps 5 --no-cpu || exit 1
JFSX_KS_STREAM=0 $S line ks0_ingest --mem host --steps 5 --no-cpu
