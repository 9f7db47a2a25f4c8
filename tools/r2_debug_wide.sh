export TMPDIR=/tmp
O=gpurun_out/dbg; mkdir -p $O
timeout -k 10 200 python tools/debug_wide.py > $O/new.log 2>&1; cat $O/new.log | grep variant
SBO_LIB=safe_bayesian_optimization_amd/lib/libsbo_base.so timeout -k 10 200 python tools/debug_wide.py > $O/base.log 2>&1; cat $O/base.log | grep variant
