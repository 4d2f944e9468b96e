#!/bin/bash
# round-3 (session 2): k_dog_peaks XCD mapping, k_dog_zconv prefetch depth / tap interleave (experiment builds)
export TMPDIR=/tmp
O=gpurun_out/r3z4
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_PEAKS_XCD=1" "SPIMDECON_DOG_PEAKS_XCD=0" "SPIMDECON_LIB=exp/libspimdecon_ilv.so" "SPIMDECON_LIB=exp/libspimdecon_pd5.so" "SPIMDECON_LIB=exp/libspimdecon_pd13.so" "SPIMDECON_LIB=exp/libspimdecon_pd5n.so" "SPIMDECON_DOG_PEAKS_XCD=1 B=1" || exit 2
