#!/bin/bash
# round 6 (v): the legacy simultaneous-update mode (lrsim_*) against its oracle, the
# one-rank RCCL all-reduce path, and a kernel trace of one C2-sized run
export TMPDIR=/tmp
O=gpurun_out/r6v
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lrsim.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -12 $O/tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -u tools/lrsim_bench.py --shape 512 512 512 --views 4 --iters 3 > $O/bench_1.log 2>&1; rc=$?; tail -4 $O/bench_1.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/lrsim_bench.py --shape 512 512 512 --views 4 --iters 2 > $O/kt.log 2>&1; rc=$?; tail -2 $O/kt.log; [ $rc = 0 ] || exit 1
f=$(find $O/kt -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv && head -14 $O/kernel_stats.csv
echo done-r6v
