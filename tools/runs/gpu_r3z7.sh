#!/bin/bash
# round-3 (session 2): L = 1050 x tiles with 40 threads per row pair (SPIMDECON_XTR=40): parity, C3 A/B
export TMPDIR=/tmp
O=gpurun_out/r3z7
mkdir -p $O
SPIMDECON_XTR=40 timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py -k "pad_policies" -x -q --timeout 250 --timeout-method thread > $O/tests.log 2>&1 || exit 1
for v in 40 0 40 0; do
  SPIMDECON_XTR=$v timeout -k 10 300 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3_$v.log 2>&1 || exit 2
  tail -1 $O/c3_$v.log >> $O/c3_$v.jsonl
done
