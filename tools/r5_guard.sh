#!/bin/bash
# Round 5: the inverse accuracy guard's tests, the re-pinned ill-conditioned
# tests, the sliced-inverse tests, then a C4 bench line (fit cost of the guard).
export TMPDIR=/tmp
O=gpurun_out/r5guard; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc; }
step guard 900 python -u -m pytest tests/test_gpu_invcheck.py tests/test_gpu_parity.py -k "invcheck or sliced or guard or ill_conditioned or length_scale or nondefault or recursive_inverse or overlap" -x -v -s --timeout 300 --timeout-method thread
step bench 400 python bench.py --no-cpu --no-regimes --steps 20
