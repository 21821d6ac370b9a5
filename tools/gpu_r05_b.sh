#!/bin/bash
# Round 5: radix-7 sizes (every 2·3·5·7-smooth N of the general engine) and the reference-run
# radix-7 fixtures, plus the constraints / mode-limit tests.
set -o pipefail
O=gpurun_out/r05/${1:-b}
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_constraints.py -x -v --timeout 300 --timeout-method thread > $O/tests_parity.txt 2>&1
