#!/bin/bash
# round 5 (z7): k_dog_peaks rows per wave (kDpkY 4 = main, 6, 8): kernel-trace A/B, alternated
# twice, then the DoG tests on the winner candidate dpk8
export TMPDIR=/tmp
O=gpurun_out/r5z7
mkdir -p $O
for k in 1 2; do
  for v in main dpk6 dpk8; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/${v}_$k -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $O/${v}_$k.log 2>&1 || exit 1
    python3 - $O/${v}_$k/k_kernel_stats.csv $v $k <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_dog_peaks" in r["Name"]:
        print(sys.argv[2], sys.argv[3], "peaks avg %.1f us" % (float(r["AverageNs"]) / 1e3))
PY
  done
done
SPIMDECON_LIB=exp/libspimdecon_dpk8.so timeout -k 10 400 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 300 --timeout-method thread > $O/tests_dpk8.log 2>&1; echo "dpk8 tests rc=$?"; tail -1 $O/tests_dpk8.log
echo done-z7
