#!/bin/bash
# round 6 (y): the whole -m gpu suite and the smoke at HEAD (legacy mode with device groups)
export TMPDIR=/tmp
O=gpurun_out/r6y
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations 10 > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit 1; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -1 $O/smoke.log; [ $rc = 0 ] || exit 1
echo done-r6y
