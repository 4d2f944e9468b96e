#!/bin/bash
# round-3: DoG two-plane steps (tests + A/B), z-pass tile width A/B, C4 at size, exchange accounting, full bench
export TMPDIR=/tmp
O=gpurun_out/r3e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_ZSTEP=2" "SPIMDECON_DOG_ZSTEP=2 SPIMDECON_DOG_ZCHUNK=128" "SPIMDECON_DOG_ZSTEP=1 SPIMDECON_DOG_ZCHUNK=128" || exit 2
for v in 64 32; do
  SPIMDECON_ZCHUNK=$v timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong-line --no-default-mode > $O/bench_zc$v.log 2>&1 || exit 3
done
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py::test_c4_timepoint_8view_768 tests/test_gpu_multidevice.py::test_c3_strong_decomposition_exchange_accounting -x -v -s --durations=0 --timeout 580 --timeout-method thread > $O/tests.log 2>&1 || exit 4
timeout -k 10 400 python3 bench.py > $O/bench.log 2>&1 || exit 5
