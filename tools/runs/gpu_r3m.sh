#!/bin/bash
# round-3: k_dog_z with a brick-layout access pattern (experiment build, values wrong)
export TMPDIR=/tmp
O=gpurun_out/r3m
mkdir -p $O
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_dz3.so SPIMDECON_BENCH_NOCHECK=1" "SPIMDECON_LIB=exp/libspimdecon_dz3.so SPIMDECON_DOG_XCD=0 SPIMDECON_BENCH_NOCHECK=1" || exit 2
