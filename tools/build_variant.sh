#!/bin/bash
# Build an experimental variant of libptyx.so: tools/build_variant.sh <name> [extra hipcc flags...]
# (ptyrad_amd/lib/var/libptyx_<name>.so, with its own build id; load it with PTYX_LIB=<path>)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
mkdir -p "$R/ptyrad_amd/lib/var"
cd "$R" && python -c "
import sys
from ptyrad_amd.csrc.build import build
build(out='ptyrad_amd/lib/var/libptyx_$name.so', extra=sys.argv[1:], verbose=False)" "$@"
echo "$R/ptyrad_amd/lib/var/libptyx_$name.so"
