#!/bin/bash
# A/B builds of one kernel source: variants/<name>.so = the in-tree objects
# with <src> recompiled under extra -D flags.  Usage:
#   tools/build_variants.sh <src.hip> name1:"-DX=1 -DY=2" name2:"..."
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/zarr_amd/csrc
SRC=$1; shift
make -s -C "$C" >/dev/null
mkdir -p "$R/variants"
base=$(basename "$SRC" .hip)
for spec in "$@"; do
  name=${spec%%:*}; defs=${spec#*:}
  d=$R/variants/obj_$name; mkdir -p "$d"
  /opt/rocm/bin/hipcc -O3 -fPIC -std=c++17 --offload-arch=gfx950 -munsafe-fp-atomics -I"$C" $defs -c "$C/$SRC" -o "$d/$base.o" &
done
wait
for spec in "$@"; do
  name=${spec%%:*}; d=$R/variants/obj_$name
  objs=$(ls "$C"/build/*.o | grep -v "/$base.o$")
  /opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "$R/variants/$name.so" $objs "$d/$base.o"
  echo "built variants/$name.so"
done
