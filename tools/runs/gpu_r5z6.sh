#!/bin/bash
# round 5 (z6): test_gpu_rl.py alone after load() imports torch before the library
# (gpu_r5z4/z5: that process aborted at exit with a double free when the library
# was loaded before torch)
export TMPDIR=/tmp
O=gpurun_out/r5z6
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_rl.log 2>&1
echo "rl rc=$?"; tail -2 $O/tests_rl.log
echo done-z6
