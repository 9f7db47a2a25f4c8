#!/bin/bash
# Round 5: guard + re-pinned + sliced-inverse tests, the pair sweep's tests and
# its lpsc-box A/B, a C4 bench line.
export TMPDIR=/tmp
O=gpurun_out/r5combo; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-600; [ $rc -eq 0 ] || exit $rc; }
step pair 600 python -u -m pytest tests/test_gpu_parity.py -k "precise_sweep_matches_oracle or kstar_table_chunks or pair_sweep or int8_mfma or warmup or diagnostic_build" -x -v -s --timeout 300 --timeout-method thread
OZ_KERNELS="3 4" step ab 600 python -u tools/r4_oz_ab.py 16384 1024
step guard 900 python -u -m pytest tests/test_gpu_invcheck.py tests/test_gpu_parity.py -k "invcheck or sliced or guard or ill_conditioned or length_scale or nondefault or recursive_inverse or overlap" -x -v -s --timeout 300 --timeout-method thread
step bench 400 python bench.py --no-cpu --no-regimes --steps 20
