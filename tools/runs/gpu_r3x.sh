#!/bin/bash
# round-3: k_dog_z test stage cost split: no neighbour LDS reads / no NaN bookkeeping / neither
export TMPDIR=/tmp
O=gpurun_out/r3x
mkdir -p $O
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_xnoread.so $N" "SPIMDECON_LIB=exp/libspimdecon_xnonan.so $N" "SPIMDECON_LIB=exp/libspimdecon_xboth.so $N" "SPIMDECON_DOG_XCD=1 A=1" || exit 2
