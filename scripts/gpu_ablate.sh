set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
B="python3 bench.py --blocks 2048 --steps 5 --warmup 1 --no-cpu --verify 0"
for v in base nocrc noghash noaes noaes_nocrc noghash_nocrc; do
  case $v in
    base) lib=juicefs_amd/libjfsx.so; extra="";;
    nocrc) lib=juicefs_amd/libjfsx.so; extra="--crc none";;
    noghash) lib=juicefs_amd/_build/libjfsx_GHASH.so; extra="";;
    noghash_nocrc) lib=juicefs_amd/_build/libjfsx_GHASH.so; extra="--crc none";;
    noaes) lib=juicefs_amd/_build/libjfsx_AES.so; extra="";;
    noaes_nocrc) lib=juicefs_amd/_build/libjfsx_AES.so; extra="--crc none";;
  esac
  JFSX_LIB=$lib timeout -k 10 120 $B $extra > gpurun_out/abl_$v.log 2>&1 || { echo "$v failed"; tail -3 gpurun_out/abl_$v.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/abl_$v.log').read().strip().splitlines()[-1]); print('$v', d['value'], d['roofline']['kernel_avg_ms'])"
done
