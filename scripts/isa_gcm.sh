# ISA summary of gcm_main<seal, CRC gen> for a build variant: round-loop mix and spill ops.
# usage: bash scripts/isa_gcm.sh [extra hipcc -D flags...]
set -e
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
src=$(pwd)/juicefs_amd/csrc/jfsx_gcm.hip; inc=$(pwd)/include; (cd $tmp && /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 "$@" -I$inc -c $src --save-temps -o g.o 2>/dev/null)
awk '/^_ZN4jfsx10gcm_main_kILb0ELi1ELi1EEEvPKNS_4TaskEPKNS_6BlkDevEPKNS_8GcmSchedEPjSA_NS_9DevTablesE:/,/s_endpgm/' $tmp/jfsx_gcm-hip-amdgcn-amd-amdhsa-gfx950.s > $tmp/m.s
python3 - $tmp/m.s <<'PY'
import re, sys
L = open(sys.argv[1]).read().splitlines()
# innermost loop = first label tagged Depth=3 (or deepest)
hdr = [i for i, l in enumerate(L) if 'Loop Header: Depth=' in l]
deep = max(hdr, key=lambda i: int(re.search(r'Depth=(\d+)', L[i]).group(1)))
lab = None
for j in range(deep, -1, -1):
    m = re.match(r'^(\.LBB\d+_\d+):', L[j])
    if m: lab = m.group(1); break
end = max(i for i, l in enumerate(L) if re.search(r's_(cbranch_\w+|branch)\s+' + re.escape(lab) + r'\b', l))
body = [l for l in L[deep:end + 1] if re.match(r'^\s+[sv]_|^\s+(ds|global|scratch|buffer|flat)_', l)]
spill = lambda ls: sum(1 for l in ls if re.search(r'scratch_|v_readlane|v_writelane', l))
print("round loop: %d instrs, %d bitop3, %d mov, %d spill ops" % (len(body), sum('v_bitop3' in l for l in body),
      sum('v_mov' in l for l in body), spill(body)))
allins = [l for l in L if re.match(r'^\s+[sv]_|^\s+(ds|global|scratch|buffer|flat)_', l)]
print("kernel: %d instrs, %d spill ops" % (len(allins), spill(allins)))
PY
rm -rf $tmp
