#!/bin/bash
# round-3 (session 2): 4 row pairs per x tile at L = 1050 / 800 (SPIMDECON_XTP=4): parity, C3 and C4 A/B
export TMPDIR=/tmp
O=gpurun_out/r3z8
mkdir -p $O
SPIMDECON_XTP=4 timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py -k "pad_policies or global_twiddles" -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for v in 4 8 4 8; do
  SPIMDECON_XTP=$v timeout -k 10 300 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3_$v.log 2>&1 || exit 2
  tail -1 $O/c3_$v.log >> $O/c3_$v.jsonl
  SPIMDECON_XTP=$v timeout -k 10 300 python3 bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$v.log 2>&1 || exit 3
  tail -1 $O/c4_$v.log >> $O/c4_$v.jsonl
done
