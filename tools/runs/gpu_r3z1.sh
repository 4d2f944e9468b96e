#!/bin/bash
# round-3 (session 2): z-pass access-pattern microbenchmark, then z-pass knob A/B on the bench
export TMPDIR=/tmp
O=gpurun_out/r3z1
mkdir -p $O
timeout -k 10 120 ./tools/zpattern_bench > $O/zpattern.txt 2>&1 || exit 1
tools/ab.sh $O/ab "-" "SPIMDECON_ZCHUNK=64" "SPIMDECON_ZSTAG_GROUP=4" "SPIMDECON_ZSTAG_GROUP=16" "SPIMDECON_ZCHUNK=16" || exit 2
