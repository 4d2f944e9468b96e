#!/bin/bash
# round 4 (b): the fused y-z-y pass -- parity tests, then the bench line and its kernel trace
export TMPDIR=/tmp
O=gpurun_out/r4b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -k "fused_yzy" -x -v --timeout 200 --timeout-method thread > $O/yzy_tests.log 2>&1
rc=$?
tail -5 $O/yzy_tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_configs.py -k "c2_4view_512 or c3_decomposition" tests/test_gpu_multidevice.py tests/test_gpu_golden.py -x -q --timeout 300 --timeout-method thread > $O/cfg_tests.log 2>&1
rc=$?
tail -3 $O/cfg_tests.log
[ $rc -eq 0 ] || exit 2
timeout -k 10 300 python3 -u bench.py --steps 10 --no-cpu-baseline --no-strong-line > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/kt.log 2>&1 || exit 4
cp $(ls $O/kt/*/k_kernel_stats.csv $O/kt/k_kernel_stats.csv 2>/dev/null | head -1) $O/kernel_stats.csv
# A/B on the same box: column passes (YZY=0), the fused pass with 8 and 12 planes per step
tools/ab.sh $O/ab "SPIMDECON_YZY=0" "-" "SPIMDECON_YZY_G=12" || exit 5
for f in $O/ab/ab_*.json; do python3 -c "import json,sys; d=json.load(open('$f')); print('$f', d['value'], d['ms_per_step'])"; done
