#!/bin/bash
# round-3: k_dog_z with the peak test but no DoG store (10); stores issued but all out of range (11)
export TMPDIR=/tmp
O=gpurun_out/r3t
mkdir -p $O
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_dz10.so $N" "SPIMDECON_LIB=exp/libspimdecon_dz11.so $N" "SPIMDECON_LIB=exp/libspimdecon_dz4.so $N" "SPIMDECON_DOG_XCD=1 A=1" || exit 2
