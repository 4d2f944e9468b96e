#!/bin/bash
# round 6 (g): voxel batches of the 2100 update wave tiles (main: 2 float4 per row with
# Tikhonov = 5 round trips per tile; vb5: 2 round trips; vb9: 1, 156 VGPRs fp16, still 3
# waves per SIMD).  Prediction: C5 update 2.82 -> ~2.6 ms if the serial batch round trips
# are exposed; neutral if the other 8 waves of the CU already hide them
export TMPDIR=/tmp
O=gpurun_out/r6g
mkdir -p $O
for v in vb5 vb9; do
SPIMDECON_LIB=exp/libspimdecon_$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py -x -q -k "x_tiles_2100" --timeout 250 --timeout-method thread > $O/tests_$v.log 2>&1; rc=$?; tail -1 $O/tests_$v.log; [ $rc = 0 ] || exit 1
done
for k in 1 2 3; do
  for v in main vb5 vb9; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --c5-rank --steps 4 --warmup 1 > $O/c5_${v}_$k.json 2> $O/c5_${v}_$k.err || { echo "c5 $v failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c5_${v}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c5 $v $k value %.1f quotient %.3f update %.3f' % (d['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms']))"
  done
done
echo done-r6g
