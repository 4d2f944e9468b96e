#!/bin/bash
# round 4 (d): the C4 back-to-back test with per-stage digests
export TMPDIR=/tmp
O=gpurun_out/r4d
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py::test_c4_two_timepoints_back_to_back_equal_fresh_process -x -q --timeout 800 --timeout-method thread > $O/c4x2.log 2>&1
rc=$?
grep -E "^E |passed|failed" $O/c4x2.log | head -12
exit $rc
