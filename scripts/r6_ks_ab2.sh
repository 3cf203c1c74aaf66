# Repeat of the keysetup-stream A/B at 256 KiB and 1 MiB, alternating, plus a
# kernel trace of the 64 KiB line with the keysetup stream on.
set -u
t=${1:-r6x}
S="bash scripts/suite.sh $t"
A="--mode agg --threads 20 --buffers heap --agg-crc seg --no-cpu --warmup-seconds 3 --agg-op seal"
for rep in a b; do
  for sz in 262144:100 1048576:30; do
    b=${sz%%:*}; n=${sz##*:}
    $S line ks1_${b}_$rep $A --block-bytes $b --steps $n || exit 1
    JFSX_KS_STREAM=0 $S line ks0_${b}_$rep $A --block-bytes $b --steps $n || exit 1
  done
done
$S prof ks1_64k $A --block-bytes 65536 --steps 20 --warmup-seconds 1
