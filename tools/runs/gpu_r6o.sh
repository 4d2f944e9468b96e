#!/bin/bash
# round 6 (o): the 1050-point y pass (C3, C5) on 8-column tiles at two blocks per CU with
# the two halves of each 16-column band on one XCD (SPIMDECON_YPAIR=1) against one 16-column
# block per CU.  The round-5 8-column tiles (0.892 -> 1.098 ms) put the halves on different
# XCDs, so both L2s fetched every 128-B segment.  Prediction: y 0.88 -> 0.80-0.84 ms if
# the L2 sharing works (C3 / C5 +2-4 %), else as round 5 (slower)
export TMPDIR=/tmp
O=gpurun_out/r6o
mkdir -p $O
SPIMDECON_YPAIR=1 timeout -k 10 400 python -u -m pytest tests/test_gpu_rl.py -x -q -k "engine_pad_policies or x_tiles_2100" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc = 0 ] || exit 1
for k in 1 2; do
  for yp in 0 1; do
    SPIMDECON_YPAIR=$yp timeout -k 10 240 python3 bench.py --no-cpu-baseline --strong --steps 4 --warmup 1 --no-default-mode --no-strong-line > $O/c3_$yp_$k.json 2> $O/c3_${yp}_$k.err || { echo "c3 failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c3_$yp_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3 ypair=$yp $k value %.1f y %.3f z %.3f q %.3f u %.3f' % (d['value'], k['y_pass']['avg_ms'], k['z_convolve']['avg_ms'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms']))"
    SPIMDECON_YPAIR=$yp timeout -k 10 240 python3 bench.py --no-cpu-baseline --c5-rank --steps 4 --warmup 1 > $O/c5_$yp_$k.json 2> $O/c5_${yp}_$k.err || { echo "c5 failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c5_$yp_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c5 ypair=$yp $k value %.1f y %.3f' % (d['value'], k['y_pass']['avg_ms']))"
  done
done
echo done-r6o
