#!/bin/bash
# One bench line per BASELINE config geometry on one GPU (gpurun): OUT/<name>.json
# usage: tools/bench_configs.sh OUT [names...]   (default: all)
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
declare -A CFG=(
  [c2_4view_512]="--views 4 --size 512"
  [c3_1024x1024x512]="--shape 1024 1024 512 --psftype EFFICIENT_BAYESIAN --lam 0.006"
  [c3_zslab_of8]="--shape 1024 1024 64 --psftype EFFICIENT_BAYESIAN --lam 0.006"
  [c3_yslab_of8]="--shape 1024 512 128 --psftype EFFICIENT_BAYESIAN --lam 0.006"
  [c5_fp16_slab]="--shape 2048 2048 128 --fp16 --psftype OPTIMIZATION_I --lam 0.006"
  [c4_rl_768]="--views 8 --size 768 --psftype OPTIMIZATION_I --lam 0.006"
  [v6_1024cube_2slabs]="--shape 1024 1024 1024 --local-slabs 2"
)
NAMES=${@:-c2_4view_512 c3_1024x1024x512 c3_zslab_of8 c3_yslab_of8 c5_fp16_slab c4_rl_768 v6_1024cube_2slabs}
for n in $NAMES; do
  echo "== $n: ${CFG[$n]}"
  timeout -k 10 300 python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-default-mode ${CFG[$n]} > $OUT/$n.log 2>&1 || exit $?
  tail -1 $OUT/$n.log > $OUT/$n.json
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['value'], 'Mvox/s', d['ms_per_step'], 'ms', d['config']['fft_dims_xyz'], 'roof', d['roofline']['kernel'], d['roofline']['frac'])"
done
