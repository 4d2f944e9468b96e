#!/bin/bash
# round-3 final pass 4: strong emulation with the y-split the 8-GPU run uses (C3), and 1024^3 (z)
export TMPDIR=/tmp
O=gpurun_out/r3m4
mkdir -p $O
for shape in "1024 1024 512" "1024 1024 1024"; do
  tag=$(echo $shape | tr ' ' x)
  for n in 1 2 4 8; do
    timeout -k 10 300 python3 -u bench.py --strong --shape $shape --local-slabs $n --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode --no-timing --no-strong-line > $O/${tag}_n$n.log 2>&1 || exit 2
    tail -1 $O/${tag}_n$n.log > $O/${tag}_n$n.json
  done
done
