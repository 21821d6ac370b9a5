#!/bin/bash
# One PMC pass of VALU-utilisation counters on the c2 bench (k_fused3): VALUBusy =
# SQ_ACTIVE_INST_VALU (quad-cycles, summed over SIMDs) / CU_NUM / GRBM_GUI_ACTIVE.
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
O=$R/gpurun_out/${1:-valu}
shift || true
mkdir -p $O
export TMPDIR=/tmp
cd /tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CU_CYCLES SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INST_CYCLES_SALU GRBM_GUI_ACTIVE \
  --output-format csv -d $O/p -o pmc -- python3 $R/bench.py --steps 1 --warmup 1 --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err
python3 - "$O" <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
f = glob.glob(O + "/p/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
disp = collections.defaultdict(set)
for r in csv.DictReader(open(f)):
    k = r["Kernel_Name"]
    if "k_fused3" not in k and "k_s" not in k: continue
    acc[k][r["Counter_Name"]] += float(r["Counter_Value"])
    disp[k].add(r["Dispatch_Id"])
for k, c in acc.items():
    n = len(disp[k])
    g = c["GRBM_GUI_ACTIVE"] / 8 / n   # per XCC per dispatch
    print(k[:60], "dispatches", n, {kk: "%.4g" % (v / n) for kk, v in c.items()})
    print("   VALUBusy %.1f%%  (ACTIVE_INST_VALU*4/(4 SIMD*256 CU*GRBM/XCC))" % (100 * c["SQ_ACTIVE_INST_VALU"] / n * 4 / (1024 * g)))
    print("   VALU issue %.1f%% of SIMD cycles (INSTS_VALU*4/(1024*GRBM/XCC))" % (100 * c["SQ_INSTS_VALU"] / n * 4 / (1024 * g)))
PY
