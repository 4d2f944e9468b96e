#!/bin/bash
# round-3: k_dog_z prefetch depth 12 / 16 (does the DoG store's cost come from the vmcnt coupling?)
export TMPDIR=/tmp
O=gpurun_out/r3s
mkdir -p $O
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_pd12.so" "SPIMDECON_LIB=exp/libspimdecon_pd16.so" "SPIMDECON_LIB=exp/libspimdecon_dz1pd16.so $N" "SPIMDECON_DOG_XCD=1 A=1" || exit 2
