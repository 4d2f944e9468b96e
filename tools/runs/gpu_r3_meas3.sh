#!/bin/bash
# round-3 final pass 3: the C4 pipeline (8 views x 768^3 x 4 timepoints) and the C3 strong emulation
export TMPDIR=/tmp
O=gpurun_out/r3m3
mkdir -p $O
timeout -k 10 400 python3 -u tools/c4_pipeline.py > $O/c4.log 2>&1 || exit 1
grep '^{' $O/c4.log | tail -1 > $O/c4.json
for n in 1 2 4 8; do
  timeout -k 10 300 python3 -u bench.py --strong --shape 1024 1024 512 --local-slabs $n --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode --no-timing --no-strong-line > $O/c3_n$n.log 2>&1 || exit 2
  tail -1 $O/c3_n$n.log > $O/c3_n$n.json
done
