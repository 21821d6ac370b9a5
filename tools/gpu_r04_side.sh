#!/bin/bash
# Side-stream branches in the register engines' calls (DESIGN §8 default cadence): correctness
# (step-graph, split, register-engine parity tests), then recon_step at ga = 1 with and without
# them (PTYX_NO_SIDE_STREAMS=1), c2 geometry and the tBL_WSe2 demo geometry.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT="$R/gpurun_out/${1:-r04m}"
mkdir -p "$OUT"
cd "$R"
timeout -k 10 400 python -u -m pytest tests/test_gpu_stepgraph.py tests/test_gpu_split.py tests/test_gpu_parity.py \
  -q -x --timeout 200 --timeout-method thread -k "not every_smooth and not mixed_radix" > "$OUT/tests.txt" 2>&1
echo "tests: $(tail -1 "$OUT/tests.txt")"
for side in on off; do
  env_=""; [ "$side" = off ] && export PTYX_NO_SIDE_STREAMS=1 || unset PTYX_NO_SIDE_STREAMS
  timeout -k 10 200 python -u tools/bench_recon.py --ga 1 --iters 2 > "$OUT/recon_c2_$side.jsonl" 2> "$OUT/recon_c2_$side.err"
  echo "c2 ga1 side=$side: $(tail -1 "$OUT/recon_c2_$side.jsonl")"
  timeout -k 10 200 python -u tools/bench_recon.py --ga 1 --iters 2 --pmodes 6 --slices 6 > "$OUT/recon_tbl_$side.jsonl" 2> "$OUT/recon_tbl_$side.err"
  echo "tbl ga1 side=$side: $(tail -1 "$OUT/recon_tbl_$side.jsonl")"
done
