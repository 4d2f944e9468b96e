#!/bin/bash
# Round-end measurement refresh on one GPU box: full GPU test suite, bench line,
# kernel trace, PMC traffic, DoG bench + trace, C4 pipeline.  usage: tools/refresh.sh OUTDIR
set -o pipefail
OUT=$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 600 --timeout-method thread > $OUT/gpu_tests.log 2>&1 &&
tools/measure.sh $OUT/m &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/dogkt -o k --output-format csv -- python3 tools/dog_bench.py --reps 3 --device-only > $OUT/dog_bench.log 2>&1 &&
timeout -k 10 400 python3 tools/c4_pipeline.py > $OUT/c4.log 2>&1
