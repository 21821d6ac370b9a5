#!/bin/bash
# Build a single-N experimental variant of libptyx.so: tools/build_variant.sh <name> [extra hipcc flags...]
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/build/var"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fno-slp-vectorize -fPIC -shared -DPTYX_ONLY_N=128 -I "$R/include" "$@" \
  -o "$R/build/var/libptyx_$name.so" "$R/ptyrad_amd/csrc/ptyx_kernels.hip" "$R/ptyrad_amd/csrc/ptyx_constraints.hip" "$R/ptyrad_amd/csrc/ptyx_ingest.hip"
echo "$R/build/var/libptyx_$name.so"
