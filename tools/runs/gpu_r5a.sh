#!/bin/bash
# round 5 (a): C5 rank-slab bench + kernel trace, fresh PMC passes at HEAD for the C3 (1050)
# and C5 (2100) x tiles
export TMPDIR=/tmp
O=gpurun_out/r5a
mkdir -p $O
timeout -k 10 400 python3 -u bench.py --c5-rank --steps 3 --warmup 1 > $O/c5.log 2>&1 || exit 1
tail -1 $O/c5.log > $O/c5.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c5kt -o k --output-format csv -- python3 bench.py --c5-rank --steps 2 --warmup 1 --no-cpu-baseline --no-timing > $O/c5kt.log 2>&1 || exit 2
timeout -k 10 700 tools/pmc_engine.sh $O/pmc1050 --strong || exit 3
timeout -k 10 700 tools/pmc_engine.sh $O/pmc_c5 --c5-rank || exit 4
echo done
