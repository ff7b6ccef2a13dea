#!/bin/bash
# Builds A/B variants of the product library for kernel experiments:
#   tools/variants.sh NAME "-DFLAG=1 ..." [NAME "FLAGS" ...]
# -> carnd-path-planning-project_amd/ppamd/libppamd_var_NAME.so (selected with PPAMD_LIB=...).
# Time them on the GPU with tools/variants_bench.sh.
set -e
PKG=$(cd "$(dirname "$0")/../carnd-path-planning-project_amd" && pwd)
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
make -C "$PKG" -s ppamd/libppamd.so
while [ $# -ge 2 ]; do
  name=$1; flags=$2; shift 2
  mkdir -p "$PKG/build/var_$name"
  $HIPCC --offload-arch=gfx950 -O3 -ffp-contract=off -fPIC -std=c++17 $flags -c \
      -o "$PKG/build/var_$name/pp_eval.o" "$PKG/csrc/pp_eval.hip" &
done
wait
for d in "$PKG"/build/var_*/; do
  name=$(basename "$d"); name=${name#var_}
  [ "$d/pp_eval.o" -nt "$PKG/ppamd/libppamd_var_$name.so" ] || continue
  $HIPCC --offload-arch=gfx950 -shared -fPIC -o "$PKG/ppamd/libppamd_var_$name.so" "$d/pp_eval.o" \
      "$PKG"/build/pp_codec_dev.o "$PKG"/build/pp_codec.o "$PKG"/build/pp_server.o -lpthread
  echo "built libppamd_var_$name.so"
done
