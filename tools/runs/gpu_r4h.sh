#!/bin/bash
# round 4 (h): engine classes at the C4 and C3 geometries (pitch 1054 at 1050), the
# strong-scaling emulation, the DoG bench and the C4 pipeline
export TMPDIR=/tmp
O=gpurun_out/r4h
mkdir -p $O
timeout -k 10 300 python3 bench.py --size 768 --views 8 --ksize 31 --psftype OPTIMIZATION_I --lam 0.006 --steps 3 --warmup 1 --no-cpu-baseline --no-strong-line --no-default-mode > $O/c4.log 2>&1 || exit 1
tail -1 $O/c4.log > $O/c4.json
timeout -k 10 300 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode > $O/c3.log 2>&1 || exit 2
tail -1 $O/c3.log > $O/c3.json
tools/strong_emulation.sh $O/strong > $O/strong.txt 2>&1 || exit 3
timeout -k 10 300 python3 -u tools/dog_bench.py > $O/dog.log 2>&1 || exit 4
grep '^{' $O/dog.log | tail -1 > $O/dog.json
timeout -k 10 400 python3 -u tools/c4_pipeline.py > $O/c4p.log 2>&1 || exit 5
grep '^{' $O/c4p.log | tail -1 > $O/c4p.json
