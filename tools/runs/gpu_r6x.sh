#!/bin/bash
# round 6 (x): the legacy mode's device groups (repeated ids on one GPU) and the rest of its tests
export TMPDIR=/tmp
O=gpurun_out/r6x
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lrsim.py -x -v --timeout 120 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -14 $O/tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 200 python -u tools/lrsim_bench.py --shape 512 512 512 --views 4 --iters 3 > $O/bench_1.log 2>&1; rc=$?; tail -1 $O/bench_1.log; [ $rc = 0 ] || exit 1
echo done-r6x
