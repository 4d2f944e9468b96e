#!/bin/bash
# round 6 (i): 1050 update x tiles as wave tiles (one wave, one row pair, the whole voxel
# row in one batch: 124 VGPRs, 16 waves per CU as now) against the 4-pair block tiles
# (3 voxel batches).  Prediction (the 2100 result: batches were the exposed round trips):
# C3 update 2.32 -> ~2.1 ms, C3 +3 %; the r6b 1050 wave tiles (batches of 2) measured 2.36
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
SPIMDECON_LIB=exp/libspimdecon_wu1050.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rl.py -x -q -k "tikhonov_update_tiles or engine_pad_policies" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc = 0 ] || exit 1
for k in 1 2 3; do
  for v in main wu1050; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --strong --steps 4 --warmup 1 --no-default-mode --no-strong-line > $O/c3_${v}_$k.json 2> $O/c3_${v}_$k.err || { echo "c3 $v failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c3_${v}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3 $v $k value %.1f quotient %.3f update %.3f' % (d['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms']))"
  done
done
echo done-r6i
