#!/bin/bash
# PMC passes (profiles/collect_pmc.sh) for the c2 bench and the N = 256 stripe engine (c5, c3).
#   tools/gpu_pmc.sh <tag>
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
TAG=${1:-pmc}
OUT="$R/gpurun_out/$TAG"
mkdir -p "$OUT"
cd "$R"
bash profiles/collect_pmc.sh "$OUT/c2" > "$OUT/c2.log" 2>&1
python3 profiles/summarize_pmc.py "$OUT/c2" "$OUT/pmc_c2.json" > "$OUT/pmc_c2.txt"
echo "c2 pmc ok"
for c in c5 c3; do
  bash profiles/collect_pmc.sh "$OUT/$c" --config $c --patterns 4096 > "$OUT/$c.log" 2>&1
  python3 profiles/summarize_pmc.py "$OUT/$c" "$OUT/pmc_$c.json" > "$OUT/pmc_$c.txt"
  echo "$c pmc ok"
done
