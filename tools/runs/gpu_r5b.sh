#!/bin/bash
# round 5 (b): after pruning the measured-slower paths -- the RL / DoG / multi-device / legacy
# GPU tests, then the default bench line
export TMPDIR=/tmp
O=gpurun_out/r5b
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_dog.py tests/test_gpu_multidevice.py tests/test_gpu_legacy.py tests/test_gpu_golden.py -m gpu -x -q -rA --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 -u bench.py --steps 10 --no-cpu-baseline > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log > $O/bench.json
echo done
