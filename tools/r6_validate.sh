export TMPDIR=/tmp
O=gpurun_out/r6a; mkdir -p $O
step() { local name=$1 lim=$2; shift 2; echo "== $name $(date +%T)"; timeout -k 10 $lim "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -3 $O/$name.log; [ $rc -eq 0 ] || exit $rc; }


step cost 300 python tools/dump_c4_cost.py
step fit_outer 400 python tools/fit_timing.py --n 2048 8192 16384 --outer 512 1024 --reps 4
step bench_c4 400 python bench.py
