#!/bin/bash
# round-3: k_dog_z without its per-plane barrier (experiment build, wrong results): the barrier's cost
export TMPDIR=/tmp
O=gpurun_out/r3w
mkdir -p $O
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_LIB=exp/libspimdecon_nobar.so SPIMDECON_BENCH_NOCHECK=1" "SPIMDECON_DOG_XCD=1 A=1" "SPIMDECON_LIB=exp/libspimdecon_nobar.so SPIMDECON_BENCH_NOCHECK=1 A=1" || exit 2
