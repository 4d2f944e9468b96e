#!/bin/bash
# round 5 (r): 4-pair update tiles at 540 too (u540: 540 headline) and 4-pair quotient tiles
# at 1050 without the image prefetch (q4: C3) vs main; alternated twice on one box
export TMPDIR=/tmp
O=gpurun_out/r5r
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main u540; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/b540_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/b540_${v}_$k.log > $O/b540_${v}_$k.json
done
for v in main q4; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/b540_*.json $O/c3_*.json
echo done-r
