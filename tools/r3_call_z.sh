#!/bin/bash
# round 3: the parity file with the large-batch append test, headline tests, smoke
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_headline.py > gpurun_out/r3c_gpu_tests.log 2>&1 || exit 11
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r3c_smoke.log 2>&1 || exit 12
