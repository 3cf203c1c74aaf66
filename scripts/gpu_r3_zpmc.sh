# PMC instruction mix and wait split of the zstd block-parallel kernel (1024
# text objects, one step).  usage: bash scripts/gpu_r3_zpmc.sh <tag>
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/$1
mkdir -p $out
export TMPDIR=/tmp
A="--mode unzstd --blocks 1024 --steps 1 --warmup 0 --no-cpu --verify 0"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE -d $out/pmc_a -o run --output-format csv -- python3 bench.py $A > $out/pmc_a.log 2>&1 || { echo "pmc a failed"; tail -3 $out/pmc_a.log; exit 1; }
echo "pmc a ok"
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES -d $out/pmc_b -o run --output-format csv -- python3 bench.py $A > $out/pmc_b.log 2>&1 || { echo "pmc b failed"; tail -3 $out/pmc_b.log; exit 1; }
echo "pmc b ok"
python3 - $out <<'PY'
import csv, glob, sys
for d in ("pmc_a", "pmc_b"):
    rows = []
    for f in glob.glob(sys.argv[1] + "/" + d + "/**/*counter_collection.csv", recursive=True):
        rows += list(csv.DictReader(open(f)))
    agg = {}
    for r in rows:
        if "zstd_decompress_par" in r["Kernel_Name"]:
            agg[r["Counter_Name"]] = agg.get(r["Counter_Name"], 0) + float(r["Counter_Value"])
    print(d, {k: "%.4g" % v for k, v in sorted(agg.items())})
PY
