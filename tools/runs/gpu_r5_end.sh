#!/bin/bash
# round 5 end: the whole -m gpu suite and smoke() at HEAD, then the C4 pipeline's stage times
export TMPDIR=/tmp
O=gpurun_out/r5end
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --durations=20 --timeout 600 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
tail -1 $O/smoke.log
timeout -k 10 400 python3 -u tools/c4_pipeline.py > $O/c4p.log 2>&1 || exit 3
grep '^{' $O/c4p.log | tail -1 > $O/c4p.json
python3 -c "
import json; d=json.load(open('$O/c4p.json'))
print('c4p', d['total_s'], [(t['t'], t['s'], {k: round(v, 1) for k, v in t['stage_ms'].items() if k in ('detect', 'prepare_inputs', 'extract_psf', 'rl_setup', 'rl_iterations')}) for t in d['timepoints']])"
echo done-end
