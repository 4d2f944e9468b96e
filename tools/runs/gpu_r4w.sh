#!/bin/bash
# round 4 (w): z pass with the zero outer taps of 2 KC - 1 plane kernels skipped at compile time
# (k_zdmc KD = 1; C4's 31-plane PSFs) vs SPIMDECON_ZKD=0: z-pass parity, the C4 timepoint test, then C4 A/B
export TMPDIR=/tmp
O=gpurun_out/r4w
mkdir -p $O
SPIMDECON_ZKD=1 timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_scale.py -x -q -k "z_pass or long_columns or c4_timepoint or engine_matches" --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log
[ $rc -eq 0 ] || exit 1
i=0
for v in 1 0 1 0; do  # (1: KD variants, 0: default)
  SPIMDECON_ZKD=$v timeout -k 10 300 python3 -u bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4_$i.log 2>&1 || exit 2
  tail -1 $O/c4_$i.log > $O/c4_$i.json
  python3 -c "import json; d=json.load(open('$O/c4_$i.json')); k=d['kernel_ms']; print('C4 ZKD=$v', d['value'], d['ms_per_step'], 'z', k['z_convolve']['avg_ms'])"
  i=$((i+1))
done
