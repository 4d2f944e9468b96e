#!/bin/bash
# round-3 (session 2): k_dog_zconv chunk length A/B (planes per block)
export TMPDIR=/tmp
O=gpurun_out/r3z10
mkdir -p $O
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_ZC_CHUNK=256" "SPIMDECON_DOG_ZC_CHUNK=384" "SPIMDECON_DOG_ZC_CHUNK=768" "SPIMDECON_DOG_ZC_CHUNK=192" "SPIMDECON_DOG_ZC_CHUNK=384 B=1" "SPIMDECON_DOG_ZC_CHUNK=256 B=1" || exit 2
