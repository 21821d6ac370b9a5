#!/bin/bash
# Round 5: tBL default-cadence trace (tools/gpu_r05_e.sh) then the whole GPU suite.
set -o pipefail
O=gpurun_out/r05/${1:-f}
mkdir -p $O
bash tools/gpu_r05_e.sh ${1:-f}/trace &&
timeout -k 10 900 python -u -m pytest tests/ -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests_gpu.txt 2>&1
