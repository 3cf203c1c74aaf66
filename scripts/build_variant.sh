# Build juicefs_amd/_build/libjfsx_<V>.so: the named source files with extra -D
# flags, linked with the default build's other objects (run make first).
# usage: bash scripts/build_variant.sh <V> "<sources, e.g. jfsx_gcm.hip jfsx_api.cpp>" <defines...>
set -eu
cd "$(dirname "$0")/../juicefs_amd"
V=$1; SRCS=$2; shift 2
objs=$(ls _build/*.o | grep -v "_var_")
vobjs=""
for SRCF in $SRCS; do
  objs=$(echo "$objs" | grep -v "/$SRCF.o")
  sched=""
  case $SRCF in jfsx_gcm.hip|jfsx_chacha.hip) sched="-mllvm -amdgpu-sched-strategy=iterative-ilp";; esac
  /opt/rocm/bin/hipcc -x hip --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-function -Wno-unused-variable $sched "$@" -I../include -c csrc/$SRCF -o _build/_var_${V}_$SRCF.o
  vobjs="$vobjs _build/_var_${V}_$SRCF.o"
done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o _build/libjfsx_$V.so.tmp $objs $vobjs
mv -f _build/libjfsx_$V.so.tmp _build/libjfsx_$V.so
