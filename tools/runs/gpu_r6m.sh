#!/bin/bash
# round 6 (m): PMC passes of the shipping kernels at the long lengths -- the C5 rank slab
# (2100 wave tiles) and C3 on one GPU (1050 tiles)
export TMPDIR=/tmp
O=gpurun_out/r6m
mkdir -p $O
bash tools/pmc_engine.sh $O/c5 --c5-rank && python3 tools/pmc_summary.py $O/c5 > $O/c5.md || { echo "c5 pmc failed"; exit 1; }
cat $O/c5.md
bash tools/pmc_engine.sh $O/c3 --strong && python3 tools/pmc_summary.py $O/c3 > $O/c3.md || { echo "c3 pmc failed"; exit 1; }
cat $O/c3.md
echo done-r6m
