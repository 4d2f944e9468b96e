#!/bin/bash
# round-3 (session 2): the DoG tests incl. the split-vs-fused agreement test
export TMPDIR=/tmp
O=gpurun_out/r3z9
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_dog.py -x -v --timeout 300 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
