#!/bin/bash
# round-3: z-pass tile width A/B, C4 at size, exchange accounting, full default bench line
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
for v in 64 32; do
  SPIMDECON_ZCHUNK=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong-line --no-default-mode > $O/bench_zc$v.log 2>&1 || exit 1
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py::test_c4_timepoint_8view_768 tests/test_gpu_multidevice.py::test_c3_strong_decomposition_exchange_accounting -x -v -s --durations=0 --timeout 580 --timeout-method thread > $O/tests.log 2>&1 || exit 2
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || exit 3
