#!/bin/bash
# round 6 (p): x tiles in descending row order (xrev).  The y-inverse pass writes the planes
# in ascending z, so the last ~256 MB it wrote (the Infinity Cache) are the high planes; the x
# tiles read rows ascending and reach them last.  Descending, they read them first; the x
# pass then leaves the low planes hot for the ascending forward y pass.  Prediction: x passes
# -3..-6 % (up to 20 % of their spectra reads served by the MALL), headline +1..2 %
export TMPDIR=/tmp
O=gpurun_out/r6p
mkdir -p $O
SPIMDECON_LIB=exp/libspimdecon_xrev.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_multidevice.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc = 0 ] || exit 1
for k in 1 2 3; do
  for v in main xrev; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 10 --no-strong-line > $O/h_${v}_$k.json 2> $O/h_${v}_$k.err || { echo "h failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/h_${v}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; dm=d['default_mode']
print('h $v $k value %.1f default %.1f q %.3f u %.3f y %.3f z %.3f' % (d['value'], dm['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms'], k['y_pass']['avg_ms'], k['z_convolve']['avg_ms']))"
  done
done
for v in main xrev; do
  L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
  SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --strong --steps 4 --warmup 1 --no-default-mode --no-strong-line > $O/c3_${v}.json 2> $O/c3_${v}.err || { echo "c3 failed"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/c3_${v}.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3 $v value %.1f q %.3f u %.3f y %.3f' % (d['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms'], k['y_pass']['avg_ms']))"
done
echo done-r6p
