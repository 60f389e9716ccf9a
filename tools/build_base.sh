#!/bin/bash
# Builds the library from a git revision (default HEAD) into tools/lib<name>_diag.so for same-box A/B
# timing against the working tree (diagnostic).  usage: bash tools/build_base.sh [rev] [name] [flags...]
set -e
cd "$(dirname "$0")/.."
REV=${1:-HEAD}; NAME=${2:-base}; shift 2 || true
T=$(mktemp -d)
git archive "$REV" mi-bminet_amd/csrc include | tar -x -C "$T"
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function \
  -mllvm -disable-promote-alloca-to-lds "$@" -shared -o tools/lib${NAME}_diag.so "$T/mi-bminet_amd/csrc/mibminet.hip"
rm -rf "$T"
ls -la tools/lib${NAME}_diag.so
