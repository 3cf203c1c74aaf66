# Round-6 host-memory lines (per-object calls in the reference's shapes, on
# pageable heap memory), each with its same-run CPU baseline.
# usage: bash scripts/r6_host_lines.sh <tag>
set -u
t=${1:-r6}
S="bash scripts/suite.sh $t line"
A="--mode agg --threads 20 --steps 10"
$S heap_seal $A --buffers heap --agg-op seal --agg-crc seg &&
$S heap_seal_both $A --buffers heap --agg-op seal --agg-crc both &&
$S heap_open $A --buffers heap --agg-op open --agg-crc seg &&
$S heap_open_both $A --buffers heap --agg-op open --agg-crc both &&
$S pinned_seal $A --agg-op seal --agg-max-mb 16 &&
$S heap_checksum $A --agg-op checksum &&
$S heap_verify $A --agg-op verify &&
$S readat_shrink $A --agg-op readat --level shrink --algo chacha20poly1305 &&
$S readat_extend $A --agg-op readat --level extend --algo chacha20poly1305
