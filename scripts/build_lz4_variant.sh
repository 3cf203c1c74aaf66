# Build juicefs_amd/_build/libjfsx_<name>.so with jfsx_lz4.hip compiled under
# extra -D flags (timing experiments only; the other objects from make).
# usage: bash scripts/build_lz4_variant.sh <name> "<defs>"
set -eu
cd "$(dirname "$0")/../juicefs_amd"
make -s
H="/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I../include -Icsrc"
$H $2 -c csrc/jfsx_lz4.hip -o _build/lz4_$1.o
OBJS=$(ls _build/*.o | grep -v '_build/lz4_' | grep -v jfsx_lz4.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _build/libjfsx_$1.so $OBJS _build/lz4_$1.o
