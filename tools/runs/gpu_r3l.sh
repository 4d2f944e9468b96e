#!/bin/bash
# round-3: k_dog_xy XCD-contiguous tiles; k_dog_z cost split (no test / no convolution builds)
export TMPDIR=/tmp
O=gpurun_out/r3l
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XY_XCD=1" "SPIMDECON_DOG_XY_XCD=0" "SPIMDECON_LIB=exp/libspimdecon_dz1.so" "SPIMDECON_LIB=exp/libspimdecon_dz2.so" || exit 2
