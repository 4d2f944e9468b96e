#!/bin/bash
# round 4 (r): y-pass prefetch at every length (SPIMDECON_YPF=2) vs the default on the 540 headline
# (bench only: gpu_r4p.sh's parity step passed, 78 tests), then the refresh's measurement half
export TMPDIR=/tmp
O=gpurun_out/r4p
mkdir -p $O
i=0
for v in 2 1 2 1 2 1; do
  SPIMDECON_YPF=$v timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/h_$i.log 2>&1 || exit 2
  tail -1 $O/h_$i.log > $O/h_$i.json
  python3 -c "import json; d=json.load(open('$O/h_$i.json')); k=d['kernel_ms']; dm=d['default_mode']; print('540 YPF=$v', d['value'], d['ms_per_step'], 'y', k['y_pass']['avg_ms'], 'default', dm['value'])"
  i=$((i+1))
done
bash tools/runs/gpu_r4_final.sh meas
