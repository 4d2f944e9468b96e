#!/bin/bash
# round 4 (u): z pass in 1024-thread blocks (SPIMDECON_ZOPT=6: 32-column tiles, OPT 6, 16 waves per CU)
# vs the default 512-thread plans: z-pass parity under it, then C4 and 540, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4u
mkdir -p $O
SPIMDECON_ZOPT=6 timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -x -q -k "z_pass or long_columns or engine_matches or mvdeconvolution_matches" --timeout 300 --timeout-method thread > $O/tests_6.log 2>&1
rc=$?
tail -1 $O/tests_6.log
[ $rc -eq 0 ] || exit 1
i=0
for v in 0 6 0 6; do
  if [ $v = 0 ]; then L=""; else L="SPIMDECON_ZOPT=$v"; fi
  env $L timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$i.log 2>&1 || exit 2
  tail -1 $O/c4_$i.log > $O/c4_$i.json
  python3 -c "import json; d=json.load(open('$O/c4_$i.json')); k=d['kernel_ms']; print('C4 ZOPT=$v', d['value'], d['ms_per_step'], 'z', k['z_convolve']['avg_ms'])"
  i=$((i+1))
done
for v in 0 6 0 6; do
  if [ $v = 0 ]; then L=""; else L="SPIMDECON_ZOPT=$v"; fi
  env $L timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line --no-default-mode > $O/h_$i.log 2>&1 || exit 3
  tail -1 $O/h_$i.log > $O/h_$i.json
  python3 -c "import json; d=json.load(open('$O/h_$i.json')); k=d['kernel_ms']; print('540 ZOPT=$v', d['value'], d['ms_per_step'], 'z', k['z_convolve']['avg_ms'])"
  i=$((i+1))
done
