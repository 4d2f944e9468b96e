#!/bin/bash
# round 4 (s): x tiles with occupancy-aware launch bounds (xt_minw) and the quotient's image
# prefetch for rows of up to 7 float4 per lane (L = 800) -- default -- vs SD_XT_QPF7=0
# (exp/libspimdecon_q0.so): parity (incl. the y-pass prefetch bit-identity test), then C4, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4s
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
i=0
for v in new q0 new q0; do
  if [ $v = new ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_$v.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$i.log 2>&1 || exit 2
  tail -1 $O/c4_$i.log > $O/c4_$i.json
  python3 -c "import json; d=json.load(open('$O/c4_$i.json')); k=d['kernel_ms']; print('C4 $v', d['value'], d['ms_per_step'], 'upd', k['x_update']['avg_ms'], 'quot', k['x_quotient']['avg_ms'], 'y', k['y_pass']['avg_ms'])"
  i=$((i+1))
done
