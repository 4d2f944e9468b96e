#!/bin/bash
# round 4 (j): Tikhonov update voxel batches at TR = 32 (540 headline, 800 C4): default
# (all KV float4 at 540, 4 at 800) vs 2 (t2) vs 3 (t3), same box, interleaved
export TMPDIR=/tmp
O=gpurun_out/r4j
mkdir -p $O
i=0
for v in base t2 t3 base t2 t3; do
  if [ $v = base ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_$v.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/h_${v}_$i.log 2>&1 || exit 1
  tail -1 $O/h_${v}_$i.log > $O/h_${v}_$i.json
  python3 -c "import json; d=json.load(open('$O/h_${v}_$i.json')); k=d['kernel_ms']; dm=d['default_mode']; print('540 $v', d['value'], d['ms_per_step'], k['x_update']['avg_ms'], 'default', dm['value'], dm['kernel_ms']['x_update']['avg_ms'])"
  i=$((i+1))
done
for v in base t2 t3; do
  if [ $v = base ]; then L=""; else L="SPIMDECON_LIB=exp/libspimdecon_$v.so"; fi
  env $L timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$v.log 2>&1 || exit 2
  tail -1 $O/c4_$v.log > $O/c4_$v.json
  python3 -c "import json; d=json.load(open('$O/c4_$v.json')); k=d['kernel_ms']; print('800 $v', d['value'], d['ms_per_step'], k['x_update']['avg_ms'])"
done
