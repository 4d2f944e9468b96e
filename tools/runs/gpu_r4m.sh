#!/bin/bash
# round 4 (m): z-pass access pattern (no compute) at the plane geometries of 540^3 (P 536,
# 540 x 272 elements), C4's 800 (P 798, 800 x 416) and C3's 1050 (P 536, 1050 x 528, rounded down to a multiple of 64)
export TMPDIR=/tmp
O=gpurun_out/r4m
mkdir -p $O
timeout -k 10 120 ./tools/zpattern_bench 536 146880 quick > $O/zp_540.txt 2>&1 || exit 1
timeout -k 10 120 ./tools/zpattern_bench 798 332800 quick > $O/zp_800.txt 2>&1 || exit 2
timeout -k 10 120 ./tools/zpattern_bench 536 554368 quick > $O/zp_1050.txt 2>&1 || exit 3
cat $O/zp_540.txt $O/zp_800.txt $O/zp_1050.txt
