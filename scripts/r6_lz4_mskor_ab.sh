# LZ4 compressor: the large-input table's high bits written by one ds_mskor_b32 (default) or an
# and / or atomic pair (libjfsx_MSK0.so, -DJFSX_LZ4_MSKOR=0); GPU LZ4 parity first, then the 4096-block
# text and random lines alternating on one box
set -u
t=${1:-r6lz}
out=gpurun_out/suite_$t
mkdir -p $out
timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lz4.py tests/test_compress_contract.py -m gpu -x -q --timeout 120 --timeout-method thread > $out/pytest_lz4.log 2>&1 || { tail -5 $out/pytest_lz4.log; exit 1; }
tail -1 $out/pytest_lz4.log
S="bash scripts/suite.sh $t line"
for rep in a b; do
  $S text_new_$rep --mode lz4 --blocks 4096 --steps 5 --warmup 1 --no-cpu || exit 1
  JFSX_LIB=juicefs_amd/_build/libjfsx_MSK0.so $S text_old_$rep --mode lz4 --blocks 4096 --steps 5 --warmup 1 --no-cpu || exit 1
done
$S random_new --mode lz4 --lz4-data random --blocks 4096 --steps 5 --warmup 1 --no-cpu || exit 1
JFSX_LIB=juicefs_amd/_build/libjfsx_MSK0.so $S random_old --mode lz4 --lz4-data random --blocks 4096 --steps 5 --warmup 1 --no-cpu
