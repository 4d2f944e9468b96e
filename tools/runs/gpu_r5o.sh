#!/bin/bash
# round 5 (o): x tiles whose DFT-phase waves are rotated per block (rotA: by blockIdx / 256,
# rotB: by blockIdx) so that the waves left idle by the phases land on different SIMDs in
# different blocks, vs main; 540 headline, C3, C4; alternated twice on one box
export TMPDIR=/tmp
O=gpurun_out/r5o
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main rotA rotB; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/b540_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/b540_${v}_$k.log > $O/b540_${v}_$k.json
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 2
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
  SPIMDECON_LIB=$L timeout -k 10 300 $T --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --no-strong-line > $O/c4_${v}_$k.log 2>&1 || exit 3
  tail -1 $O/c4_${v}_$k.log > $O/c4_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/b540_*.json $O/c3_*.json $O/c4_*.json
echo done-o
