#!/bin/bash
# round-3 (session 2): split DoG z stage with the register-only test pass k_dog_peaks:
# bit-exactness, then A/B (rows per lane, test chunk, the ring test, the fused kernel)
export TMPDIR=/tmp
O=gpurun_out/r3z3
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
SPIMDECON_DOG_PEAKS_Y=8 timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 250 --timeout-method thread > $O/dog_tests_y8.log 2>&1 || exit 2
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_SPLIT=1" "SPIMDECON_DOG_PEAKS_Y=8" "SPIMDECON_DOG_PEAKS_ZC=128" "SPIMDECON_DOG_PEAKS_ZC=32" "SPIMDECON_DOG_SPLIT=0" || exit 3
