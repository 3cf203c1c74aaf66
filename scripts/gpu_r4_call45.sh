# Round-4 call 45: LZ4 compressor candidate extensions (LEXT: a short match
# from the probe's own 24-byte load, no count_and_back) against the default:
# parity on LEXT, then the 16 GiB text line A/B, same box.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4aj; mkdir -p $out
export TMPDIR=/tmp
L=juicefs_amd/_build/libjfsx_LEXT.so
JFSX_LIB=$L timeout -k 10 300 python3 -u -m pytest tests/test_gpu_lz4.py tests/test_compress_contract.py -q --timeout 120 --timeout-method thread > $out/t.log 2>&1
rc=$?; echo "LEXT tests rc $rc: $(tail -1 $out/t.log)"; [ $rc -ne 0 ] && { grep -E "FAILED|Error" $out/t.log | head -5; exit 1; }
run() { local name=$1; shift; timeout -k 10 300 python3 bench.py --no-cpu --verify 4 --blocks 4096 --mode lz4 "$@" > $out/ab_$name.json 2> $out/ab_$name.err || { echo "$name failed"; tail -3 $out/ab_$name.err; return 1; }; python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], 'value', d['value'], 'ms', d['ms_per_step'])" $out/ab_$name.json $name; }
run main && JFSX_LIB=$L run ext && run main2 && JFSX_LIB=$L run ext2 && run rmain --lz4-data random && JFSX_LIB=$L run rext --lz4-data random
