#!/bin/bash
# round 4 (l): x-tile DFT lane map AM = 2 (xt_amap, default) vs AM = 0 (exp/libspimdecon_am0.so):
# x-tile parity first, then 540 headline / default mode, C3 strong (1050) and C4 (800), same box, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4l
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
i=0
for v in am2 am0 am2 am0; do
  if [ $v = am2 ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_$v.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline > $O/h_${v}_$i.log 2>&1 || exit 2
  tail -1 $O/h_${v}_$i.log > $O/h_${v}_$i.json
  python3 -c "import json; d=json.load(open('$O/h_${v}_$i.json')); k=d['kernel_ms']; dm=d['default_mode']; st=d['strong']; print('$v 540', d['value'], d['ms_per_step'], 'upd', k['x_update']['avg_ms'], 'quot', k['x_quotient']['avg_ms'], 'default', dm['value'], 'C3', st['value'], st['ms_per_step'])"
  i=$((i+1))
done
for v in am2 am0; do
  if [ $v = am2 ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_$v.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3_$v.log 2>&1 || exit 3
  tail -1 $O/c3_$v.log > $O/c3_$v.json
  python3 -c "import json; d=json.load(open('$O/c3_$v.json')); k=d['kernel_ms']; print('$v C3', d['value'], d['ms_per_step'], 'upd', k['x_update']['avg_ms'], 'quot', k['x_quotient']['avg_ms'])"
  env $L timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$v.log 2>&1 || exit 4
  tail -1 $O/c4_$v.log > $O/c4_$v.json
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); k=d['kernel_ms']; print('$v C4', d['value'], d['ms_per_step'], 'upd', k['x_update']['avg_ms'], 'quot', k['x_quotient']['avg_ms'])"
done
