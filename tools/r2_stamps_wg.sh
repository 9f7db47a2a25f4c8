export TMPDIR=/tmp
O=gpurun_out/stamps2; mkdir -p $O
D=safe_bayesian_optimization_amd/lib/libsbo_diag.so
SBO_LIB=$D timeout -k 10 200 python tools/x3_stamps.py --config C4 --save $O/wg_c4.npy > $O/c4.log 2>&1 && tail -3 $O/c4.log &&
SBO_LIB=$D SBO_LVL_FORCE=0 timeout -k 10 200 python tools/x3_stamps.py --config C4 --save $O/wg_c4f0.npy > $O/c4f0.log 2>&1 && tail -3 $O/c4f0.log
