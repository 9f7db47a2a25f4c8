#!/bin/bash
# Round 5 bundle: the pipelined pair sweep (tests + A/B), then fit latency,
# the C4 fit trace, the shard emulation and the hyper-parameter calibration.
bash tools/r5_pair2.sh || exit $?
bash tools/r5_fit.sh
