#!/bin/bash
# Strong-scaling estimate on ONE GPU (the 8-GPU run is the driver's): BASELINE configs[2]
# (6-view 1024x1024x512, EFFICIENT_BAYESIAN lambda 0.006) and the north star's 6-view
# 1024^3, each split into N y- (C3) or z-slabs (1024^3) run as N local slabs of one
# session; per-GPU time ~ ms_per_step / N (halo exchange excluded: a compute-only
# projection).  usage: tools/strong_emulation.sh OUT
set -o pipefail
OUT=$1
mkdir -p $OUT
for shape in "1024 1024 512" "1024 1024 1024"; do
  tag=$(echo $shape | tr ' ' x)
  for n in 1 2 4 8; do
    timeout -k 10 300 python3 bench.py --strong --shape $shape --local-slabs $n --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode --no-timing --no-strong-line > $OUT/${tag}_n$n.log 2>&1 || exit $?
    tail -1 $OUT/${tag}_n$n.log > $OUT/${tag}_n$n.json
    python3 -c "import json; d=json.load(open('$OUT/${tag}_n$n.json')); c=d['config']; print('$tag', $n, d['ms_per_step'], d['value'], c['slabs'], c['fft_dims_xyz'])"
  done
done
