#!/bin/bash
# round-3: PMC traffic of k_dog_z variants (default, 64x16 boxes, no test, no test + no store)
export TMPDIR=/tmp
O=gpurun_out/r3q
mkdir -p $O
tools/pmc_dog.sh $O/def SPIMDECON_DOG_XCD=1 || exit 1
tools/pmc_dog.sh $O/by16 SPIMDECON_DOG_Z_BY=16 || exit 1
tools/pmc_dog.sh $O/dz1 SPIMDECON_LIB=exp/libspimdecon_dz1.so SPIMDECON_BENCH_NOCHECK=1 || exit 1
tools/pmc_dog.sh $O/dz4 SPIMDECON_LIB=exp/libspimdecon_dz4.so SPIMDECON_BENCH_NOCHECK=1 || exit 1
