#!/bin/bash
# round 5 (f): x-tile A/B on one box -- C5 rank slab: main (PF, pipelined update) vs pfq (+
# the quotient's image prefetch under PF); C3: main vs qpf64 (64-thread image prefetch) vs
# pipe1 / pipe2 (64-thread update pipeline, without / with the early first batch); the 540
# headline; C3's 8-slab exchange window with the neighbour halo planes skipped by the x
# passes; stamps at 540 / 2100; parity of the main build at 1050 / 2100 and the slabs
export TMPDIR=/tmp
O=gpurun_out/r5f
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for v in main pfq trx trxq coltrx trxall; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --c5-rank > $O/c5_$v.log 2>&1 || exit 1
  tail -1 $O/c5_$v.log > $O/c5_$v.json
done
for v in main qpf64 pipe1 pipe2 trx trxq coltrx trxall; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_$v.log 2>&1 || exit 2
  tail -1 $O/c3_$v.log > $O/c3_$v.json
done
python3 tools/ab_summary.py $O/c5_*.json $O/c3_*.json
timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/b540.log 2>&1 || exit 3
tail -1 $O/b540.log > $O/b540.json
SPIMDECON_LIB=$PWD/exp/libspimdecon_pf540.so timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/b540_pf540.log 2>&1 || exit 3
tail -1 $O/b540_pf540.log > $O/b540_pf540.json
timeout -k 10 300 python3 -u bench.py --strong --local-slabs 8 --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3x8.log 2>&1 || exit 4
tail -1 $O/c3x8.log > $O/c3x8.json
python3 tools/ab_summary.py $O/b540.json $O/b540_pf540.json $O/c3x8.json
timeout -k 10 700 python -u -m pytest tests/test_gpu_scale.py tests/test_gpu_rl.py tests/test_gpu_multidevice.py tests/test_gpu_configs.py -k "c5_rank or c5_decomposition or tikhonov or y_split or c3_decomposition or device_groups" -m gpu -x -q --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
echo done-f
