#!/bin/bash
# builds tools/split_chain_bench (gfx950) next to its source; the binary travels with the tree
set -e
cd "$(dirname "$0")"
/opt/rocm/bin/hipcc -O3 -std=c++17 --offload-arch=gfx950 split_chain_bench.hip -o split_chain_bench
