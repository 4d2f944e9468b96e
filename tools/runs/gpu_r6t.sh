#!/bin/bash
# round 6 (t): the Infinity-Cache banded y-z-y schedule, re-tried on the direct z pass
# (round 2's attempt ran the fused FFT z pass).  A 540^3 spectrum is 627 MB; a band of B kx
# columns is B * 2.3 MB (64: 148 MB, 96: 221 MB) and the MALL holds 256 MB, so a band's
# y forward, z and y inverse should read HBM once and write it once (write-back permitting)
# instead of three times each.  Prediction: y + z + y per convolution 0.65 -> 0.45-0.55 ms if
# the MALL holds the band, minus ~15 launches' tails; headline +3..10 %, or slower if the
# tails dominate (round 2)
export TMPDIR=/tmp
O=gpurun_out/r6t
mkdir -p $O
SPIMDECON_BAND=64 timeout -k 10 400 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc = 0 ] || exit 1
for k in 1 2; do
  for b in 0 32 64 96; do
    SPIMDECON_BAND=$b timeout -k 10 240 python3 bench.py --no-cpu-baseline --steps 10 --no-strong-line > $O/h_${b}_$k.json 2> $O/h_${b}_$k.err || { echo "h failed"; tail -3 $O/h_${b}_$k.err; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/h_${b}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']; dm=d['default_mode']
print('h band=$b $k value %.1f default %.1f q %.3f u %.3f y %.3f z %.3f' % (d['value'], dm['value'], k['x_quotient']['avg_ms'], k['x_update']['avg_ms'], k['y_pass']['avg_ms'], k['z_convolve']['avg_ms']))"
  done
done
echo done-r6t
