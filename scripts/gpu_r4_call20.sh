# Round-4 call 20: where the zstd compressor's waves spend their cycles at
# full occupancy (4096 objects, 16 waves per CU): SQ wait / issue counters.
set -u
cd "$GRAFT_REPO_ROOT"
out=gpurun_out/r4t; mkdir -p $out
export TMPDIR=/tmp
pmc() { local name=$1 ctr=$2; shift 2; timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $ctr -d $out/pmc_$name -o run --output-format csv -- python3 bench.py --steps 1 --warmup 0 --no-cpu --verify 0 --mode zstd --blocks 4096 > $out/pmc_$name.log 2>&1 || { echo "pmc $name failed"; grep -v "^ *@" $out/pmc_$name.log | tail -3; return 1; }; python3 - $out/pmc_$name <<'PY'
import csv,glob,sys
for f in glob.glob(sys.argv[1]+'/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        if 'zstd_compress' in r.get('Kernel_Name',''): print(sys.argv[1].split('/')[-1], r['Counter_Name'], r['Counter_Value'])
PY
}
pmc sq1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU GRBM_GUI_ACTIVE" && \
pmc sq2 "SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_LDS" && \
pmc sq3 "SQ_INST_CYCLES_VMEM_RD SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
