#!/bin/bash
# round 4 (a): the C5 fp16 x-tile oracle test, the corrected streaming microbenchmark,
# PMC passes of the engine at L = 1050 (C3 on one GPU) and L = 800 (C4 geometry)
export TMPDIR=/tmp
O=gpurun_out/r4a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py::test_c5_decomposition_matches_oracle_232x256x104 tests/test_gpu_multidevice.py -x -v --timeout 300 --timeout-method thread > $O/c5_test.log 2>&1 || exit 1
timeout -k 10 180 ./tools/zpattern_bench > $O/zpattern.txt 2>&1 || exit 2
tools/pmc_engine.sh $O/pmc1050 --strong || exit 3
python3 tools/pmc_summary.py $O/pmc1050 > $O/pmc1050.md || exit 4
tools/pmc_engine.sh $O/pmc800 --shape 768 768 768 --ksize 31 --views 2 --psftype OPTIMIZATION_I || exit 5
python3 tools/pmc_summary.py $O/pmc800 > $O/pmc800.md || exit 6
