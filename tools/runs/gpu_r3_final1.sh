#!/bin/bash
# round-3 (session 2) final pass 1: the whole -m gpu suite, smoke(), the bench line and its kernel trace
export TMPDIR=/tmp
O=gpurun_out/r3f1
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --durations=15 --timeout 400 --timeout-method thread > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line > $O/kt.log 2>&1 || exit 4
cp $(ls $O/kt/*/k_kernel_stats.csv $O/kt/k_kernel_stats.csv 2>/dev/null | head -1) $O/kernel_stats.csv
