#!/bin/bash
# Register/spill report of one kernel across compile-time variants (device-only compile):
#   tools/spill_sweep.sh <kernel-name-regex> "<label>:<flags>" ...
# e.g. tools/spill_sweep.sh 'k_fused2ILi128' "base:" "nt1024:-DPTYX_FUSED_NT128=1024"
set -uo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
pat=$1; shift
tmp=$(mktemp -d)
for spec in "$@"; do
  IFS=: read -r label flags <<< "$spec"
  ( /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -I "$R/include" -DPTYX_ONLY_N=128 $flags \
      --cuda-device-only -S -o "$tmp/$label.s" "$R/ptyrad_amd/csrc/ptyx_kernels.hip" 2> "$tmp/$label.err" ) &
done
wait
for spec in "$@"; do
  IFS=: read -r label flags <<< "$spec"
  python3 - "$tmp/$label.s" "$pat" "$label" <<'EOF'
import re, sys
path, pat, label = sys.argv[1:]
try:
    txt = open(path).read()
except OSError:
    print(f"{label}: compile failed"); sys.exit(0)
for m in re.finditer(r"\.name:\s+(\S+)\n(.*?)(?=\n\s+- \.|\Z)", txt, re.S):
    name, body = m.group(1), m.group(2)
    if not re.search(pat, name):
        continue
    get = lambda k: (re.search(rf"\.{k}:\s+(\d+)", body) or [None, "?"])[1]
    print(f"{label:>14} {name[:60]:60} vgpr {get('vgpr_count'):>4} vspill {get('vgpr_spill_count'):>4} "
          f"sspill {get('sgpr_spill_count'):>3} scratch {get('private_segment_fixed_size')}")
EOF
done
rm -rf "$tmp"
