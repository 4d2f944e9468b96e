#!/bin/bash
# round 5 (z4): exit status of the RL test process on main, twice (the u540m variant's test
# process aborted at exit in gpu_r5z3.sh after all tests passed)
export TMPDIR=/tmp
O=gpurun_out/r5z4
mkdir -p $O
for k in 1 2; do
  timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$k.log 2>&1
  echo "run $k rc=$?"; tail -2 $O/tests_$k.log
done
echo done-z4
