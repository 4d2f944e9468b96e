#!/bin/bash
# round 4 (k): parity of the adopted Tikhonov batches, then the bench line
export TMPDIR=/tmp
O=gpurun_out/r4k
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_configs.py tests/test_gpu_multidevice.py -x -q --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit 1
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit 2
tail -1 $O/bench.log > $O/bench.json
python3 -c "import json; d=json.load(open('$O/bench.json')); print(d['value'], d['ms_per_step'], d['default_mode']['value'], d['strong']['value'], d['strong']['ms_per_step'])"
