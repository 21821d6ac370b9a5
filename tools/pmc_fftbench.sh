#!/bin/bash
# PMC passes over build/fftbench (kernel-level diagnosis of the FFT variants).
set -euo pipefail
R=$(cd "$(dirname "$0")/.." && pwd)
OUT=${1:-$R/gpurun_out/pmc_fft}
mkdir -p "$OUT"
export TMPDIR=/tmp
cd /tmp
i=0
for pass in "SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS GRBM_GUI_ACTIVE" \
            "SQ_INSTS_LDS SQ_INSTS_LDS_LOAD SQ_INSTS_LDS_STORE SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_LDS_UNALIGNED_STALL SQ_INSTS_VALU" \
            "SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL SQ_INST_LEVEL_LDS SQ_THREAD_CYCLES_VALU SQ_INSTS_SALU SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_MUL_F32"; do
  i=$((i + 1))
  timeout -k 10 120 rocprofv3 --pmc $pass --output-format csv -d "$OUT/pass$i" -o pmc -- "$R/build/fftbench" 50 > "$OUT/pass$i.log" 2>&1
done
echo done $i
