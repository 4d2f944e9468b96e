#!/bin/bash
# round-3: k_dog_z candidate flush through global (not flat) memory ops: the plane prefetch
# no longer drains; brick-pattern and no-test experiment builds beside it
export TMPDIR=/tmp
O=gpurun_out/r3n
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_DOG_Z_BY=16" "SPIMDECON_DOG_Z_TBL=1" "SPIMDECON_LIB=exp/libspimdecon_dz3.so SPIMDECON_BENCH_NOCHECK=1" "SPIMDECON_LIB=exp/libspimdecon_dz1.so SPIMDECON_BENCH_NOCHECK=1" || exit 2
