#!/bin/bash
# Round 5: LDS bank conflicts and instruction mix of the 512-thread FFT microbenchmark vs the
# 256-thread one (separate PMC passes, kernel trace only).
set -o pipefail
O=gpurun_out/r05/${1:-d}
mkdir -p $O build
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
hipcc --offload-arch=gfx950 -O3 -std=c++17 -I ptyrad_amd/csrc -I tools tools/regfft512bench.hip -o build/regfft512bench > $O/bench_build.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/pmc1 -o pmc1 --output-format csv -- ./build/regfft512bench 20 > $O/pmc1.txt 2>&1 &&
timeout -s KILL 90 rocprofv3 --kernel-trace --stats -d $O/kt -o kt --output-format csv -- ./build/regfft512bench 20 > $O/kt.txt 2>&1
exit 0
