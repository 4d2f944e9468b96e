#!/bin/bash
# round 5 (j): C3 (1050 tiles, spill-free after the loop removal): Tikhonov update in batches
# of 4 float4 (vb4) and the quotient's image rows loaded before the inverse transform at 64
# threads per pair (qpf64) vs main; alternated twice on one box
export TMPDIR=/tmp
O=gpurun_out/r5j
mkdir -p $O
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
for k in 1 2; do
for v in main vb4 qpf64; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 $T --strong > $O/c3_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/c3_${v}_$k.log > $O/c3_${v}_$k.json
done
done
python3 tools/ab_summary.py $O/c3_*.json
echo done-j
