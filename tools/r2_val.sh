export TMPDIR=/tmp
O=gpurun_out/v1; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }
step gpu_tests 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread
step smoke 200 python -c "import __graft_entry__ as g; g.smoke()"
step bench_c4 400 python bench.py --steps 20
echo done
