# Build juicefs_amd/_build/libjfsx_<V>.so: jfsx_crc.hip with extra -D flags,
# linked with the default build's other objects (make first).
# usage: bash scripts/build_crc_variant.sh <V> <defines...>
set -eu
cd "$(dirname "$0")/../juicefs_amd"
V=$1; shift
objs=$(ls _build/*.o | grep -v jfsx_crc.hip.o | grep -v "_crcvar_")
/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable "$@" -I../include -c csrc/jfsx_crc.hip -o _build/_crcvar_$V.o
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _build/libjfsx_$V.so $objs _build/_crcvar_$V.o
