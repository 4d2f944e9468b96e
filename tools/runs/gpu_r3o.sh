#!/bin/bash
# round-3: k_dog_z cost split: no test (1), no test + no DoG store (4), registers only (5), loads only (6), brick pattern (3)
export TMPDIR=/tmp
O=gpurun_out/r3o
mkdir -p $O
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_dz1.so $N" "SPIMDECON_LIB=exp/libspimdecon_dz4.so $N" "SPIMDECON_LIB=exp/libspimdecon_dz5.so $N" "SPIMDECON_LIB=exp/libspimdecon_dz6.so $N" "SPIMDECON_DOG_XCD=1 SPIMDECON_BENCH_NOCHECK=0" "SPIMDECON_LIB=exp/libspimdecon_dz1.so SPIMDECON_BENCH_NOCHECK=2" || exit 2
