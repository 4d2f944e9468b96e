#!/bin/bash
# round 5 (n): DoG A/B, device-resident 768^3, alternated twice on one box: main = rolling
# strips of 48 rows; s32 = strips of 32 rows at 4 blocks per CU (the x phase of a step is one
# wave-iteration per wave); zcl / s32zcl = + k_dog_zconv without the cross-step reuse of
# symmetric-tap products (148 -> 54 VGPRs); dogbase = the round-4 tiles.  DoG parity tests on
# s32zcl first.
export TMPDIR=/tmp
O=gpurun_out/r5n
mkdir -p $O
SPIMDECON_LIB=$PWD/exp/libspimdecon_s32zcl.so timeout -k 10 600 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py -m gpu -x -q -k "dog or DoG or c4" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
for k in 1 2; do
for v in main s32 zcl s32zcl dogbase; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 python3 tools/dog_bench.py > $O/dog_${v}_$k.log 2>&1 || exit 1
  grep '^{' $O/dog_${v}_$k.log | tail -1 > $O/dog_${v}_$k.json
  echo "$v $k $(python3 -c "import json; d=json.load(open('$O/dog_${v}_$k.json')); print(d['ms_device_resident'])")"
done
done
for v in s32zcl dogbase; do
  SPIMDECON_LIB=$PWD/exp/libspimdecon_$v.so timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/kt_$v.log 2>&1 || exit 3
  cp $(ls $O/kt_$v/*/k_kernel_stats.csv $O/kt_$v/k_kernel_stats.csv 2>/dev/null | head -1) $O/dog_kernel_stats_$v.csv
done
echo done-n
