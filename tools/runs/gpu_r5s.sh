#!/bin/bash
# round 5 (s): the bench's strong C3 line (run in the bench process after the 540 lines) at
# HEAD vs the round-5 measurement build (r5z, before the tile-loop removal / image prefetch /
# 4-pair update tiles): full default bench without the CPU baseline, alternated twice
export TMPDIR=/tmp
O=gpurun_out/r5s
mkdir -p $O
for k in 1 2; do
for v in main r5z; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 python3 -u bench.py --no-cpu-baseline > $O/b_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/b_${v}_$k.log > $O/b_${v}_$k.json
  python3 -c "import json; d=json.load(open('$O/b_${v}_$k.json')); print('$v $k', d['value'], d['default_mode']['value'], d['strong']['value'], d['strong']['ms_per_step'])"
done
done
echo done-s
