#!/bin/bash
# round 5 (m): DoG xy stage as rolling strips (main) vs the round-4 tiles (dogbase): the DoG
# parity tests on main, then the device-resident DoG bench alternated twice, and a kernel trace
export TMPDIR=/tmp
O=gpurun_out/r5m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py -m gpu -x -q -k "dog or DoG or c4" --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit 5
for k in 1 2; do
for v in main dogbase; do
  if [ $v = main ]; then L=""; else L=$PWD/exp/libspimdecon_$v.so; fi
  SPIMDECON_LIB=$L timeout -k 10 300 python3 tools/dog_bench.py > $O/dog_${v}_$k.log 2>&1 || exit 1
  grep '^{' $O/dog_${v}_$k.log | tail -1 > $O/dog_${v}_$k.json
  echo "$v $k $(python3 -c "import json; d=json.load(open('$O/dog_${v}_$k.json')); print(d['ms_device_resident'])")"
done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/dogkt.log 2>&1 || exit 3
cp $(ls $O/dogkt/*/k_kernel_stats.csv $O/dogkt/k_kernel_stats.csv 2>/dev/null | head -1) $O/dog_kernel_stats.csv
echo done-m
