# Round-6 per-object Encrypt (+ checksum()) on heap buffers by block size:
# where does the drop-in's per-call path stop paying?  20 callers, each line
# with its same-run CPU baseline (dataEncryptor.Encrypt + checksum() of the
# same block size on 16 host threads) and host_cpu.
# usage: bash scripts/r6_sizes.sh <tag>
set -u
t=${1:-r6s}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg"
$S size_64k $A --block-bytes 65536 --steps 400 &&
$S size_256k $A --block-bytes 262144 --steps 100 &&
$S size_1m $A --block-bytes 1048576 --steps 30 &&
$S size_ragged $A --ragged --steps 20 &&
$S size_open_64k --mode agg --threads 20 --buffers heap --agg-op open --agg-crc seg --block-bytes 65536 --steps 400
