#!/bin/bash
# round 5 (d): the whole -m gpu suite on the pruned build (PF x tiles at 2100), then (c)
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -q -rA --durations=15 --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
bash tools/runs/gpu_r5c.sh
