#!/bin/bash
# round 6 (l): what a weak-scaling rank pays for its neighbours, emulated on one GPU:
# 512^3 (no neighbour) vs 512x512x1024 as 2 local z-slabs (each one neighbour, as ranks 0
# and N-1) vs 512x512x1536 as 3 (the middle slab has two, as ranks 1..N-2); Mvox/s per slab
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
for k in 1 2; do
for c in "1 512" "2 1024" "3 1536"; do
  set -- $c
  timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-default-mode --no-strong-line --steps 6 --warmup 1 --shape 512 512 $2 --local-slabs $1 --slab-axis z > $O/w$1_$k.json 2> $O/w$1_$k.err || { echo "w$1 failed"; tail -3 $O/w$1_$k.err; exit 1; }
  python3 -c "
import json; d=json.loads(open('$O/w$1_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('slabs $1 value %.1f ms %.2f' % (d['value'], d['ms_per_step']), ' '.join('%s %.3f' % (c, k[c]['avg_ms']) for c in ('x_quotient','x_update','y_pass','z_convolve','halo_exchange','exchange_window') if c in k))"
done
done
echo done-r6l
