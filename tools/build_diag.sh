#!/bin/bash
# Builds diagnostic variants of the library: tools/lib<name>_diag.so for each "name:FLAGS" arg,
# e.g.  bash tools/build_diag.sh base: nobar:-DMIB_DIAG_NOBAR
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function \
    -mllvm -disable-promote-alloca-to-lds -DMIB_DIAG $flags -shared -o tools/lib${name}_diag.so \
    mi-bminet_amd/csrc/mibminet.hip &
done
wait
ls -la tools/*_diag.so
