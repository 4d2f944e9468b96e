#!/bin/bash
# Strong-scaling estimate on ONE GPU (the 8-GPU run is the driver's): BASELINE configs[2]
# (6-view 1024x1024x512, EFFICIENT_BAYESIAN lambda 0.006) split into N y-slabs run as N
# local slabs of one session; per-rank time ~ ms_per_step / N (halo exchange excluded).
# usage: tools/strong_emulation.sh OUT
set -o pipefail
OUT=$1
mkdir -p $OUT
for n in 1 2 4 8; do
  timeout -k 10 300 python3 bench.py --strong --local-slabs $n --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode --no-timing > $OUT/n$n.log 2>&1 || exit $?
  tail -1 $OUT/n$n.log > $OUT/n$n.json
  python3 -c "import json; d=json.load(open('$OUT/n$n.json')); print($n, d['ms_per_step'], d['config']['fft_dims_xyz'])"
done
