#!/bin/bash
# round-3: what the k_dog_z DoG store costs: stores to one plane (L2-resident), non-temporal policies
export TMPDIR=/tmp
O=gpurun_out/r3r
mkdir -p $O
N=SPIMDECON_BENCH_NOCHECK=1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_dz9.so $N" "SPIMDECON_LIB=exp/libspimdecon_nt2.so" "SPIMDECON_LIB=exp/libspimdecon_nt3.so" "SPIMDECON_LIB=exp/libspimdecon_nt18.so" "SPIMDECON_DOG_XCD=1 A=1" || exit 2
