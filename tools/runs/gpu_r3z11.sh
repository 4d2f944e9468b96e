#!/bin/bash
# round-3 (session 2): k_dog_xy without the per-value range check when min / max are the image's own
export TMPDIR=/tmp
O=gpurun_out/r3z11
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 300 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_MM_EXACT=1" "SPIMDECON_DOG_MM_EXACT=0" "SPIMDECON_DOG_MM_EXACT=1 B=1" "SPIMDECON_DOG_MM_EXACT=0 B=1" || exit 2
