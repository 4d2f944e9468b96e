#!/bin/bash
# round 6 (aa): C3's rank slab alone on one GPU (bench.py --c3-rank: 1024x128x512 y-slab,
# padded 1050x540x152 -- the geometry each GPU runs at N = 8) beside the 8-slab emulation
export TMPDIR=/tmp
O=gpurun_out/r6aa
CLASSES="c3rank c3x8 c3rank" bash tools/engine_classes.sh $O || exit 1
echo done-r6aa
