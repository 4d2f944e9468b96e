#!/bin/bash
# round-3 (session 2): per-class engine timings at the C4 (8-view 768^3, 31^3 PSF, OPTIMIZATION_I 0.006)
# and C3 (strong, one GPU) geometries
export TMPDIR=/tmp
O=gpurun_out/r3z6
mkdir -p $O
timeout -k 10 300 python3 bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4.log 2>&1 || exit 1
timeout -k 10 300 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3.log 2>&1 || exit 2
