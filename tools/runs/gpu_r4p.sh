#!/bin/bash
# round 4 (p): y-pass prefetch at every 16-column length >= 512 (SPIMDECON_YPF=2: the 540 headline's
# two-blocks-per-CU y pass too) vs the default (one-block-per-CU lengths only): parity with YPF=2,
# then the 540 headline, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
SPIMDECON_YPF=2 timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
i=0
for v in 2 1 2 1 2 1; do
  SPIMDECON_YPF=$v timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/h_$i.log 2>&1 || exit 2
  tail -1 $O/h_$i.log > $O/h_$i.json
  python3 -c "import json; d=json.load(open('$O/h_$i.json')); k=d['kernel_ms']; dm=d['default_mode']; print('540 YPF=$v', d['value'], d['ms_per_step'], 'y', k['y_pass']['avg_ms'], 'default', dm['value'])"
  i=$((i+1))
done
