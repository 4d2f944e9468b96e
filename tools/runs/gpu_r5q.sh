#!/bin/bash
# round 5 (q): Tikhonov / plain update tiles of 4 row pairs (4 blocks per CU) at 1050 (np4u)
# and at 1050 + 800 (np4u8) vs main (8 pairs); C3 and C4, alternated twice on one box; then
# the RL parity tests on np4u8
export TMPDIR=/tmp
O=gpurun_out/r5q
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main np4u; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
done
for v in main np4u8; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --no-strong-line > $O/c4_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c4_${v}_$k.log > $O/c4_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c3_*.json $O/c4_*.json
SPIMDECON_LIB=$PWD/exp/libspimdecon_np4u8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
echo done-q
