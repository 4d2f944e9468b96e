#!/bin/bash
# round 6 (w): the default bench line with the new legacy_simultaneous object (its wall
# time), and the kernel trace of the legacy mode (4 views of 512^3, additive)
export TMPDIR=/tmp
O=gpurun_out/r6w
mkdir -p $O
S=$(date +%s)
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1; rc=$?; echo "bench rc=$rc wall $(( $(date +%s) - S )) s"; [ $rc = 0 ] || { tail -5 $O/bench.log; exit 1; }
tail -1 $O/bench.log > $O/bench.json
python3 -c "
import json; d=json.load(open('$O/bench.json')); print('bench', d['value'], 'legacy', d['legacy_simultaneous'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/kt -o run --output-format csv -- python3 tools/lrsim_bench.py --shape 512 512 512 --views 4 --iters 2 > $O/kt.log 2>&1; rc=$?; tail -2 $O/kt.log; [ $rc = 0 ] || exit 1
f=$(find $O/kt -name '*kernel_stats.csv' | head -1); [ -n "$f" ] && cp "$f" $O/kernel_stats.csv
echo done-r6w
