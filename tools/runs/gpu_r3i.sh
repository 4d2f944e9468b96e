#!/bin/bash
# round-3: DoG box 32x16 (bit-exactness + A/B) and k_dog_xy persistent-grid sweep
export TMPDIR=/tmp
O=gpurun_out/r3i
mkdir -p $O
SPIMDECON_DOG_Z_BX=32 timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests_bx32.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_Z_BX=32 SPIMDECON_DOG_XY_ROUNDS=4" "SPIMDECON_DOG_Z_BX=64 SPIMDECON_DOG_XY_ROUNDS=8" "SPIMDECON_DOG_XY_ROUNDS=16" "SPIMDECON_DOG_XY_ROUNDS=2" || exit 2
