#!/bin/bash
# round 6 (a): the JNA-configuration child (no torch, /opt/rocm 7.2), the C5 rank bench,
# and the first PMC passes of the shipping persistent (PF) 2100 x tiles
export TMPDIR=/tmp
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_jna_runtime.py -x -v -s --timeout 280 --timeout-method thread > $O/jna.log 2>&1 || { echo "jna rc=$?"; tail -30 $O/jna.log; exit 1; }
tail -3 $O/jna.log
timeout -k 10 300 python3 bench.py --c5-rank --steps 4 --warmup 1 --no-cpu-baseline > $O/c5.json 2> $O/c5.err || { echo "c5 bench failed"; tail -20 $O/c5.err; exit 1; }
tail -c 1500 $O/c5.json
bash tools/pmc_engine.sh $O/pmc --c5-rank && python3 tools/pmc_summary.py $O/pmc > $O/pmc.md; echo "pmc rc=$?"
cat $O/pmc.md
echo done-r6a
