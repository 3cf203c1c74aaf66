# Round-6 final build, part B, on one box: the default and decrypt lines, the
# rocprofv3 kernel stats of the same commands, and the PMC passes (FETCH_SIZE,
# WRITE_SIZE, SQ busy counters; one counter set per run) of the seal and open
# kernels -> gpurun_out/suite_<tag>/, summarised by scripts/pmc_r3.py into
# profiles/r6/pmc_r6.json.
# usage: bash scripts/r6_final_b.sh <tag>
set -u
t=${1:-r6fb}
S="bash scripts/suite.sh $t"
SQ="SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_VALU GRBM_GUI_ACTIVE"
$S line default && $S prof default &&
$S line decrypt_gcm --mode decrypt --steps 5 --warmup 1 &&
$S prof decrypt_gcm --mode decrypt --steps 5 --warmup 1 &&
$S pmc seal_gcm__fetch FETCH_SIZE && $S pmc seal_gcm__write WRITE_SIZE &&
$S pmc open_gcm__fetch FETCH_SIZE --mode open && $S pmc open_gcm__write WRITE_SIZE --mode open &&
$S pmc seal_gcm__sq "$SQ" --blocks 1024 && $S pmc open_gcm__sq "$SQ" --blocks 1024 --mode open
