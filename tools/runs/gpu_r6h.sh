#!/bin/bash
# round 6 (h): launch bound 3 waves per SIMD for the 2100 wave tiles (w3): the fp16 quotient
# with its image prefetch goes 170 -> 162 VGPRs, 8 -> 9 waves per CU (the LDS limit), no
# spills.  Prediction: quotient 1.78 -> ~1.65 ms; update unchanged (156 VGPRs either way)
export TMPDIR=/tmp
O=gpurun_out/r6h
mkdir -p $O
SPIMDECON_LIB=exp/libspimdecon_w3.so timeout -k 10 300 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_scale.py -x -q -k "x_tiles_2100 or c5_rank_slab" --timeout 250 --timeout-method thread > $O/tests_w3.log 2>&1; rc=$?; tail -1 $O/tests_w3.log; [ $rc = 0 ] || exit 1
for k in 1 2 3; do
  for v in main w3; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --c5-rank --steps 4 --warmup 1 > $O/c5_${v}_$k.json 2> $O/c5_${v}_$k.err || { echo "c5 $v failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c5_${v}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c5 $v $k value %.1f quotient %.3f update %.3f' % (d['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms']))"
  done
done
echo done-r6h
