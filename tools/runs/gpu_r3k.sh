#!/bin/bash
# round-3: k_dog_z scalar plane index + per-plane buffer loads, 64x16 boxes (bit-exactness + A/B)
export TMPDIR=/tmp
O=gpurun_out/r3k
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
SPIMDECON_DOG_Z_BY=16 timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests_by16.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_Z_TBL=0" "SPIMDECON_DOG_Z_TBL=1" "SPIMDECON_DOG_Z_BY=16" "SPIMDECON_DOG_Z_BY=16 SPIMDECON_DOG_Z_TBL=1" || exit 2
