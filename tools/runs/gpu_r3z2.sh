#!/bin/bash
# round-3 (session 2): split DoG z stage (k_dog_zconv + k_dog_z test pass over the stored DoG):
# bit-exactness, then A/B against the fused k_dog_z and the conv chunk length
export TMPDIR=/tmp
O=gpurun_out/r3z2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_SPLIT=1" "SPIMDECON_DOG_SPLIT=0" "SPIMDECON_DOG_ZC_CHUNK=128" "SPIMDECON_DOG_ZC_CHUNK=384" "SPIMDECON_DOG_SPLIT=1 SPIMDECON_DOG_Z_BY=16" || exit 2
