#!/bin/bash
# round 4 (n): z-pass chunk configurations at C4's 800 (31-plane kernels, KC 16) and at 540:
# default plan vs SPIMDECON_ZNB=3 / ZCHUNK=16 / ZOPT=n, same box, env-selected (one build)
export TMPDIR=/tmp
O=gpurun_out/r4n
mkdir -p $O
i=0
for v in base ZNB=3 ZCHUNK=16 ZOPT=8 ZOPT=15 base; do
  if [ $v = base ]; then L=""; else L="SPIMDECON_$v"; fi
  env $L timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$i.log 2>&1 || exit 1
  tail -1 $O/c4_$i.log > $O/c4_$i.json
  python3 -c "import json; d=json.load(open('$O/c4_$i.json')); k=d['kernel_ms']; print('C4 $v', d['value'], d['ms_per_step'], 'z', k['z_convolve']['avg_ms'], 'zmodes', d.get('zpass_modes'))"
  i=$((i+1))
done
for v in base ZOPT=12 ZOPT=8 ZNB=3 base; do
  if [ $v = base ]; then L=""; else L="SPIMDECON_$v"; fi
  env $L timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line --no-default-mode > $O/h_$i.log 2>&1 || exit 2
  tail -1 $O/h_$i.log > $O/h_$i.json
  python3 -c "import json; d=json.load(open('$O/h_$i.json')); k=d['kernel_ms']; print('540 $v', d['value'], d['ms_per_step'], 'z', k['z_convolve']['avg_ms'])"
  i=$((i+1))
done
