#!/bin/bash
# round 5 final, in two calls: `tests` = the whole -m gpu suite and smoke(); `meas` = the bench
# line, its kernel trace and PMC passes, the C3 / C4 / C5-rank class lines, the C3 8-slab
# exchange window and the C4 pipeline
export TMPDIR=/tmp
O=${O:-gpurun_out/r5z}
mkdir -p $O
if [ "$1" != "meas" ]; then
  timeout -k 10 1000 python -u -m pytest tests -m gpu -q -rA --durations=20 --timeout 600 --timeout-method thread > $O/tests.log 2>&1
  rc=$?
  tail -3 $O/tests.log
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 120 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 2
  tail -1 $O/smoke.log
  exit 0
fi
timeout -k 10 500 python3 -u bench.py > $O/bench.log 2>&1 || exit 3
tail -1 $O/bench.log > $O/bench.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line > $O/kt.log 2>&1 || exit 4
cp $(ls $O/kt/*/k_kernel_stats.csv $O/kt/k_kernel_stats.csv 2>/dev/null | head -1) $O/kernel_stats.csv
tools/pmc_engine.sh $O/pmc || exit 5
DIMS=$(python3 -c "import json; print(','.join(map(str, json.load(open('$O/bench.json'))['config']['fft_dims_xyz'])))") &&
python3 tools/pmc_summary.py $O/pmc --json $O/pmc_traffic.json --dims $DIMS > $O/pmc.md
T="python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode"
timeout -k 10 300 $T --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --no-strong-line > $O/c4.log 2>&1 || exit 6
tail -1 $O/c4.log > $O/c4.json
timeout -k 10 300 $T --strong > $O/c3.log 2>&1 || exit 7
tail -1 $O/c3.log > $O/c3.json
timeout -k 10 300 $T --c5-rank > $O/c5.log 2>&1 || exit 8
tail -1 $O/c5.log > $O/c5.json
timeout -k 10 300 $T --strong --local-slabs 8 > $O/c3x8.log 2>&1 || exit 9
tail -1 $O/c3x8.log > $O/c3x8.json
python3 tools/ab_summary.py $O/bench.json $O/c4.json $O/c3.json $O/c5.json $O/c3x8.json
timeout -k 10 400 python3 -u tools/c4_pipeline.py > $O/c4p.log 2>&1 || exit 10
grep '^{' $O/c4p.log | tail -1 > $O/c4p.json
echo done-final
