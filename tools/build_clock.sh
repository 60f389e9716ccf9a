#!/bin/bash
# Builds the in-kernel clock probes (tools/clock_probe.hip) for the shipped kernel and its
# ablations: tools/clkbin_<name> for each "name:FLAGS" arg (MIB_CLOCK is always added).
set -e
cd "$(dirname "$0")/.."
for spec in "$@"; do
  name=${spec%%:*}; flags=${spec#*:}
  /opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 -Wno-unused-function -Wno-unused-result \
    -mllvm -disable-promote-alloca-to-lds -DMIB_CLOCK -DMIB_DIAG $flags -o tools/clkbin_${name} tools/clock_probe.hip &
done
wait
