# Build juicefs_amd/_build/libjfsx_<name>.so with jfsx_zstd.hip compiled under
# extra -D flags, optionally from the sources of git revision <rev> (timing
# experiments only; the other objects from make).
# usage: bash scripts/build_zstd_variant.sh <name> "<defs>" [rev]
set -eu
cd "$(dirname "$0")/../juicefs_amd"
make -s
inc=csrc
if [ $# -ge 3 ]; then
  inc=_build/zsrc_$1
  mkdir -p $inc
  for f in jfsx_zstd.h jfsx_zstd.hip; do git show $3:juicefs_amd/csrc/$f > $inc/$f; done
fi
H="/opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wno-unused-result -I../include -I$inc -Icsrc"
$H $2 -c $inc/jfsx_zstd.hip -o _build/zstd_$1.o
OBJS=$(ls _build/*.hip.o _build/*.cpp.o | grep -v jfsx_zstd.hip.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _build/libjfsx_$1.so $OBJS _build/zstd_$1.o
