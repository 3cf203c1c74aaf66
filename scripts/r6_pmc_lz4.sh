# PMC passes of the LZ4 compressor after the ds_mskor change (4096 blocks of text; one counter set per
# run), summarised with the GCM passes of r6_final_b.sh into profiles/r6/pmc_r6.json by scripts/pmc_r3.py
set -u
t=${1:-r6pl}
S="bash scripts/suite.sh $t"
SQ="SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU GRBM_GUI_ACTIVE"
A="--mode lz4 --blocks 4096"
$S pmc lz4_text__fetch FETCH_SIZE $A && $S pmc lz4_text__write WRITE_SIZE $A && $S pmc lz4_text__sq "$SQ" $A
