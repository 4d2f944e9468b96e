#!/bin/bash
# Full measurement pass on the GPU box: bench line, kernel-trace stats, PMC traffic.
# usage: tools/measure.sh OUTDIR   (then copy OUTDIR/{bench.json,kernel_stats.csv,pmc.md,pmc_traffic.json} to profiles/)
set -o pipefail
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 400 python3 bench.py > $OUT/bench.log 2>&1 && tail -1 $OUT/bench.log > $OUT/bench.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/kt -o k --output-format csv -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-legacy-line > $OUT/kt.log 2>&1 &&
cp $(ls $OUT/kt/*/k_kernel_stats.csv $OUT/kt/k_kernel_stats.csv 2>/dev/null | head -1) $OUT/kernel_stats.csv &&
tools/pmc_engine.sh $OUT/pmc &&
DIMS=$(python3 -c "import json; print(','.join(map(str, json.load(open('$OUT/bench.json'))['config']['fft_dims_xyz'])))") &&
python3 tools/pmc_summary.py $OUT/pmc --json $OUT/pmc_traffic.json --dims $DIMS > $OUT/pmc.md
