# Round-4 call 12: bisect the register-window zstd parser (JFSX_ZC_WIN bits:
# 1 search, 2 count_back, 4 literals, 8 inserts / repcode loop, 16 window reuse)
# on the byte-for-byte test that failed (text, up to 4 MiB).
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4l; mkdir -p $out
export TMPDIR=/tmp
for v in 1 2 3 7 15 17 31; do
  JFSX_LIB=juicefs_amd/_build/libjfsx_ZW$v.so timeout -k 10 200 python3 -u -m pytest "tests/test_gpu_zstdc.py::test_frames_equal_libzstd_level1" -q --timeout 120 --timeout-method thread > $out/zw${v}.log 2>&1
  rc=$?
  echo "ZW$v rc $rc: $(tail -1 $out/zw${v}.log)"
  grep -o "AssertionError: ([^)]*)" $out/zw${v}.log | head -3
  grep -o "At index [0-9]* diff" $out/zw${v}.log | head -3
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: rc $rc"; exit 1; fi
done
