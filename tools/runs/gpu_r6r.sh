#!/bin/bash
# round 6 (r): register prefetch of the next column tile in the 540 y pass (ypf540; until now
# only at one block per CU: 640-1024).  The forward y pass moves 0.66 GB of HBM for its
# 1.26 GB (Infinity-Cache hits) in 0.177 ms = 3.7 TB/s: latency-bound, not HBM-bound.
# 102 VGPRs, still 4 waves per SIMD.  Prediction: forward y 0.177 -> ~0.16 ms, inverse
# unchanged (HBM-bound at 5.9 TB/s); headline +0.5..1.3 %
export TMPDIR=/tmp
O=gpurun_out/r6r
mkdir -p $O
SPIMDECON_LIB=exp/libspimdecon_ypf540.so timeout -k 10 400 python -u -m pytest tests/test_gpu_configs.py tests/test_gpu_golden.py -x -q -k "c2_4view_512_matches or golden" --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc = 0 ] || exit 1
for k in 1 2 3; do
  for v in main ypf540; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 10 --no-strong-line > $O/h_${v}_$k.json 2> $O/h_${v}_$k.err || { echo "h failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/h_${v}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; dm=d['default_mode']
print('h $v $k value %.1f default %.1f q %.3f u %.3f y %.3f z %.3f' % (d['value'], dm['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms'], k['y_pass']['avg_ms'], k['z_convolve']['avg_ms']))"
  done
done
for v in main ypf540; do
  L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
  SPIMDECON_LIB=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/kt_$v -o k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/kt_$v.log 2>&1 || { echo "kt failed"; exit 1; }
  python3 - $O/kt_$v/k_kernel_stats.csv $v <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if "k_col2f<1, 20, 27" in r["Name"]:
        print(sys.argv[2], r["Name"][40:80], r["Calls"], "%.1f us" % (float(r["AverageNs"]) / 1e3))
PY
done
echo done-r6r
