#!/bin/bash
# round 4 (c): x-tile pitch at L = 1050 (C3 on one GPU), same box: L + 2 vs L + 4 (exp build)
export TMPDIR=/tmp
O=gpurun_out/r4c
mkdir -p $O
for v in base p4; do
  if [ $v = base ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_p4.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/strong_$v.log 2>&1 || exit 1
  tail -1 $O/strong_$v.log > $O/strong_$v.json
  python3 -c "import json; d=json.load(open('$O/strong_$v.json')); k=d['kernel_ms']; print('$v', d['value'], d['ms_per_step'], {n: k[n]['avg_ms'] for n in ('x_update','x_quotient') if n in k})"
done
timeout -k 10 180 ./tools/zpattern_bench > $O/zpattern.txt 2>&1 || exit 2
timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print('default', d['value'], d['ms_per_step'], d['config'].get('zpass_modes'))"
