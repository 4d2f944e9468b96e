#!/bin/bash
# round 6 (k): the whole -m gpu suite after the PF-tile removal, the smoke, a C5 rank and
# a headline bench line
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations 10 > $O/tests.log 2>&1; rc=$?; tail -14 $O/tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc = 0 ] || exit 1
timeout -k 10 240 python3 bench.py --no-cpu-baseline --c5-rank --steps 4 --warmup 1 > $O/c5.json 2> $O/c5.err || exit 1
python3 -c "import json; d=json.loads(open('$O/c5.json').read().strip().splitlines()[-1]); print('c5', d['value'], d['pointwise']['frac'])"
timeout -k 10 300 python3 bench.py --no-cpu-baseline > $O/h.json 2> $O/h.err || exit 1
python3 -c "import json; d=json.loads(open('$O/h.json').read().strip().splitlines()[-1]); print('headline', d['value'], d['roofline']['frac'], 'default', d['default_mode']['value'], 'strong', d['strong']['value'])"
echo done-r6k
