#!/bin/bash
# round 5 (g): C3 y pass at L = 1050 on 8-column tiles (two blocks per CU) vs 16-column
# tiles (one block per CU): main vs tx8, alternated twice on one box
export TMPDIR=/tmp
O=gpurun_out/r5g
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main tx8; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c3_*.json
echo done-g
