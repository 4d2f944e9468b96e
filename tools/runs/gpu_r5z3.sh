#!/bin/bash
# round 5 (z3): 4-pair update tiles at 540 with their own lane map (AM 3, pitch L + 12;
# modeled 579 -> 50 conflict cycles per wave) vs main (8 pairs); 540 headline alternated
# three times; then the RL parity tests on u540m
export TMPDIR=/tmp
O=gpurun_out/r5z3
mkdir -p $O
for k in 1 2 3; do
for v in main u540m; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 200 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/b540_${v}_$k.log 2>&1 || exit 1
  tail -1 $O/b540_${v}_$k.log > $O/b540_${v}_$k.json
  python3 -c "import json; d=json.load(open('$O/b540_${v}_$k.json')); print('$v $k', d['value'], d['default_mode']['value'], d['kernel_ms']['x_update']['avg_ms'], d['default_mode']['kernel_ms']['x_update']['avg_ms'])"
done
done
SPIMDECON_LIB=$PWD/exp/libspimdecon_u540m.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -m gpu -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
echo done-z3
