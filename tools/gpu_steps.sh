#!/bin/bash
# GPU session helper: each step under its own time limit; stop on any fault-like exit.
mkdir -p gpurun_out
ok() { local rc=$1; [ $rc -eq 0 ] || [ $rc -eq 1 ]; }
run() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > gpurun_out/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 gpurun_out/$name.log; ok $rc || exit $rc; }
