# Round-6 per-object ChaCha20-Poly1305 (chacha20-rsa) on heap buffers: Encrypt + checksum() at
# 4 MiB and 64 KiB with CPU baselines, and a kernel trace of the 64 KiB line
set -u
t=${1:-r6cc}
S="bash scripts/suite.sh $t"
A="--mode agg --threads 20 --buffers heap --agg-op seal --agg-crc seg --algo chacha20poly1305"
$S line chacha_seal $A --steps 10 &&
$S line chacha_open --mode agg --threads 20 --buffers heap --agg-op open --agg-crc seg --algo chacha20poly1305 --steps 10 &&
$S line chacha_64k $A --block-bytes 65536 --steps 400 &&
$S prof chacha_64k $A --block-bytes 65536 --steps 20 --warmup-seconds 1
