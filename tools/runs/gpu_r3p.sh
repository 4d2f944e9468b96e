#!/bin/bash
# round-3: k_dog_z with 64-aligned full-line DoG stores (experiment build), interleaved with the default
export TMPDIR=/tmp
O=gpurun_out/r3p
mkdir -p $O
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_dz7.so $N" "SPIMDECON_LIB=exp/libspimdecon_dz8.so $N" "SPIMDECON_DOG_XCD=1 A=1" "SPIMDECON_LIB=exp/libspimdecon_dz8.so $N A=1" || exit 2
