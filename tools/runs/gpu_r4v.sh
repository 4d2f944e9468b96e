#!/bin/bash
# round 4 (v): HEAD check -- the whole -m gpu suite, smoke(), then one bench line
export TMPDIR=/tmp
bash tools/runs/gpu_r4_final.sh tests || exit $?
O=gpurun_out/r4f
timeout -k 10 500 python3 -u bench.py > $O/bench_head.log 2>&1 || exit 3
tail -1 $O/bench_head.log > $O/bench_head.json
python3 -c "import json; d=json.load(open('$O/bench_head.json')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['default_mode']['value'], d['strong']['value'])"
