#!/bin/bash
# round 4 (i): long x tiles at L = 1050 (C3 on one GPU), same box: image prefetch in the
# quotient tile for TR = 64 (SD_XT_QPF64) and 2-float4 batches in the Tikhonov update
# (SD_XT_VB_TIK64=2), each against the default build, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4i
mkdir -p $O
i=0
for v in base qpf vb2 base qpf vb2; do
  if [ $v = base ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_$v.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/s_${v}_$i.log 2>&1 || exit 1
  tail -1 $O/s_${v}_$i.log > $O/s_${v}_$i.json
  python3 -c "import json; d=json.load(open('$O/s_${v}_$i.json')); k=d['kernel_ms']; print('$v', d['value'], d['ms_per_step'], {n: k[n]['avg_ms'] for n in ('x_update','x_quotient') if n in k})"
  i=$((i+1))
done
