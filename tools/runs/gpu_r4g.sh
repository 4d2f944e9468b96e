#!/bin/bash
# round 4 (g): the fused pass with wave-local transforms (k_yzy_wl): parity, then A/B
export TMPDIR=/tmp
O=gpurun_out/r4g
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -k "fused_yzy" -x -q --timeout 200 --timeout-method thread > $O/yzy_tests.log 2>&1
rc=$?
tail -3 $O/yzy_tests.log
[ $rc -eq 0 ] || exit 1
tools/ab.sh $O/ab "-" "SPIMDECON_YZY=1" "SPIMDECON_YZY=1 SPIMDECON_YZY_WL=0" || exit 2
for f in $O/ab/ab_*.json; do python3 -c "import json; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'], {k: v['avg_ms'] for k, v in d['kernel_ms'].items() if 'avg_ms' in v})"; done
