#!/bin/bash
# round 5 (p): 2100 (np4) and 1050 + 2100 (np4b) x tiles of 4 row pairs (np4: 67-KB tiles with global twiddles, two blocks
# of 4 waves per CU) vs 8 (one 151-KB block of 8 waves): C5 rank slab, alternated twice; then
# the C5 rank-slab test vs rocFFT on np4; C3 main vs np4b
export TMPDIR=/tmp
O=gpurun_out/r5p
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main np4; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --c5-rank > $O/c5_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/c5_${v}_$k.log > $O/c5_${v}_$k.json
done
done
for k in 1 2; do
for v in main np4b; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c5_*.json $O/c3_*.json
SPIMDECON_LIB=$PWD/exp/libspimdecon_np4.so timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q -k "c5_rank_slab or c5_full" --timeout 500 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
echo done-p
