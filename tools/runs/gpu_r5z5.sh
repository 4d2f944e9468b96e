#!/bin/bash
# round 5 (z5): exit status of the RL test process with the libraries of two earlier commits
# (bisecting the exit-time heap abort seen at HEAD in gpu_r5z4.sh)
export TMPDIR=/tmp
O=gpurun_out/r5z5
mkdir -p $O
for v in 28fe20d 5845efd; do
  SPIMDECON_LIB=$PWD/exp/libspimdecon_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests_$v.log 2>&1
  echo "$v rc=$?"; tail -2 $O/tests_$v.log
done
echo done-z5
