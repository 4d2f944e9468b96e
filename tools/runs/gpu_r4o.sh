#!/bin/bash
# round 4 (o): y-pass register prefetch of the next tile (k_col2f PF, L = 640 / 800 / 1024 at
# one block per CU) vs SPIMDECON_YPF=0: engine parity first, then the C4 geometry, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4o
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
i=0
for v in pf base pf base; do
  if [ $v = pf ]; then L=""; else L="SPIMDECON_YPF=0"; fi
  env $L timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$i.log 2>&1 || exit 2
  tail -1 $O/c4_$i.log > $O/c4_$i.json
  python3 -c "import json; d=json.load(open('$O/c4_$i.json')); k=d['kernel_ms']; print('C4 $v', d['value'], d['ms_per_step'], 'y', k['y_pass']['avg_ms'], 'z', k['z_convolve']['avg_ms'])"
  i=$((i+1))
done
for v in pf base; do
  if [ $v = pf ]; then L=""; else L="SPIMDECON_YPF=0"; fi
  env $L timeout -k 10 300 python3 -u bench.py --size 1000 --views 2 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/k_$i.log 2>&1 || exit 3
  tail -1 $O/k_$i.log > $O/k_$i.json
  python3 -c "import json; d=json.load(open('$O/k_$i.json')); k=d['kernel_ms']; print('1024 $v', d['value'], d['ms_per_step'], 'y', k['y_pass']['avg_ms'], d['config']['fft_dims_xyz'])"
  i=$((i+1))
done
