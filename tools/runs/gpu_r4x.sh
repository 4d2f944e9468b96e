#!/bin/bash
# round 4 (x): strong-scaling emulation (C3 y-slabs, 1024^3 z-slabs as N local slabs of one GPU) on the final HEAD
export TMPDIR=/tmp
O=gpurun_out/r4x
mkdir -p $O
timeout -k 10 700 tools/strong_emulation.sh $O/strong > $O/strong.txt 2>&1 || exit 1
cat $O/strong.txt
