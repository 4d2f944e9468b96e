#!/bin/bash
# round-3: the whole -m gpu suite (the round-end gate), then smoke()
export TMPDIR=/tmp
O=gpurun_out/r3suite
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --durations=15 --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
