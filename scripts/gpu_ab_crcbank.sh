# A/B on one box: GCM seal+CRC as built, without CRC, and with conflict-free
# (wrong) CRC addressing (JFSX_ABLATE_CRCBANK), 8 GiB batches, twice each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ab_crcbank
mkdir -p $out
B="python3 bench.py --blocks 2048 --steps 5 --warmup 1 --no-cpu --verify 0"
for rep in 1 2; do
for v in base nocrc crcbank; do
  case $v in
    base) lib=juicefs_amd/libjfsx.so; extra="";;
    nocrc) lib=juicefs_amd/libjfsx.so; extra="--crc none";;
    crcbank) lib=juicefs_amd/_build/libjfsx_CRCBANK.so; extra="";;
  esac
  JFSX_LIB=$lib timeout -k 10 120 $B $extra > $out/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $out/$v.$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/$v.$rep.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"
done
done
