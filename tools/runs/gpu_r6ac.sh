#!/bin/bash
# round 6 (ac): final refresh at HEAD (legacy mode, DoG tap trim, c3rank class): the whole -m gpu suite, the smoke, the
# bench line + kernel trace + PMC (tools/measure.sh), the engine classes of every geometry
export TMPDIR=/tmp
O=gpurun_out/r6ac
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations 10 > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc = 0 ] || exit 1
bash tools/measure.sh $O/m || { echo "measure failed"; exit 1; }
python3 -c "
import json; d=json.load(open('$O/m/bench.json')); print('bench', d['value'], d['ms_per_step'], d['roofline']['frac'], 'default', d['default_mode']['value'], 'strong', d['strong']['value'], 'cpu', d['cpu_baseline']['value'])"
bash tools/engine_classes.sh $O/classes || exit 1
echo done-r6ac
