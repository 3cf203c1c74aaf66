# Round-6 final build, part A: the driver's sequence (pytest -m gpu, smoke,
# default bench line), the decrypt lines (64 GiB and 2 TiB, with the GPU RSA
# unwrap on lane pairs) and the rocprofv3 kernel stats of the decrypt step.
# usage: bash scripts/r6_final_a.sh <tag>
set -u
t=${1:-r6f}
S="bash scripts/suite.sh $t"
$S tests && $S smoke && $S line default &&
$S line decrypt_gcm --mode decrypt --steps 5 --warmup 1 &&
$S line decrypt_2tib --mode decrypt --total-gib 2048 --steps 3 --warmup 1 &&
$S prof decrypt_gcm --mode decrypt --steps 5 --warmup 1 &&
$S prof default
