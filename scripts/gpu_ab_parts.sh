# Which part of gcm_main_k sets its time: as built, without CRC, without
# GHASH (wrong tags), without both (AES-CTR only), 8 GiB, twice each.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/ab_parts
mkdir -p $out
B="python3 bench.py --blocks 2048 --steps 5 --warmup 1 --no-cpu --verify 0"
for rep in 1 2; do
for v in base nocrc noghash aesonly; do
  case $v in
    base) lib=juicefs_amd/libjfsx.so; extra="";;
    nocrc) lib=juicefs_amd/libjfsx.so; extra="--crc none";;
    noghash) lib=juicefs_amd/_build/libjfsx_GHASH.so; extra="";;
    aesonly) lib=juicefs_amd/_build/libjfsx_GHASH.so; extra="--crc none";;
  esac
  JFSX_LIB=$lib timeout -k 10 120 $B $extra > $out/$v.$rep.log 2>&1 || { echo "$v failed"; tail -3 $out/$v.$rep.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('$out/$v.$rep.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"
done
done
