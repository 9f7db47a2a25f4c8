export TMPDIR=/tmp
O=gpurun_out/c5prof; mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/p -o run --output-format csv -- python bench.py --config C5 --steps 50 --no-cpu > $O/b.log 2>&1; echo rc=$?; tail -1 $O/b.log | cut -c1-300
