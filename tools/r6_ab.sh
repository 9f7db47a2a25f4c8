# round-6 A/B: the previous build (lib/libsbo_prev.so) against this one -- bitwise outputs, warm fit times,
# a kernel trace of the C4 fit; then the -m gpu suite.   bash tools/r6_ab.sh [TAG]
export TMPDIR=/tmp; O=gpurun_out/${1:-r6b}; mkdir -p $O
timeout -k 10 400 python tools/compare_libs.py safe_bayesian_optimization_amd/lib/libsbo_prev.so safe_bayesian_optimization_amd/lib/libsbo.so > $O/cmp_prev.log 2>&1; echo "cmp rc=$?"
SBO_LIB=$PWD/safe_bayesian_optimization_amd/lib/libsbo_prev.so timeout -k 10 200 python tools/fit_timing.py --n 2048 16384 --reps 4 > $O/fit_prev.log 2>&1 && timeout -k 10 200 python tools/fit_timing.py --n 2048 16384 --reps 4 > $O/fit_new.log 2>&1 && timeout -k 10 200 rocprofv3 --kernel-trace -d $O/ft4 -o run --output-format csv -- python tools/fit_timing.py --n 16384 --reps 2 > $O/ft4.log 2>&1 && timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1; echo "rc=$?"
