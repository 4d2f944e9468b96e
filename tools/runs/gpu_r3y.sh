#!/bin/bash
# round-3: k_dog_z unsigned range checks + branch-free flags (bit-exactness, A/B vs the previous build),
# and linear plane offsets (no mirror arithmetic per load; experiment build, wrong values)
export TMPDIR=/tmp
O=gpurun_out/r3y
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_nopipe.so" "SPIMDECON_LIB=exp/libspimdecon_linload.so $N" "SPIMDECON_DOG_XCD=1 A=1" "SPIMDECON_LIB=exp/libspimdecon_nopipe.so A=1" "SPIMDECON_LIB=exp/libspimdecon_linload.so $N A=1" || exit 2
