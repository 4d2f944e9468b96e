#!/bin/bash
# round-3 A/B: DoG box mapping / chunking, z-pass buffers, then the large-geometry tests
export TMPDIR=/tmp
O=gpurun_out/r3c
mkdir -p $O
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_XCD=1" "SPIMDECON_DOG_XCD=0" "SPIMDECON_DOG_XCD=0 SPIMDECON_DOG_ZCHUNK=128" "SPIMDECON_DOG_XCD=1 SPIMDECON_DOG_ZCHUNK=128" || exit 1
tools/pmc_dog.sh $O/dogpmc || exit 2
for nb in 3 2; do
  SPIMDECON_ZNB=$nb timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong-line --no-default-mode > $O/bench_znb$nb.log 2>&1 || exit 3
done
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py -k "c5_full or c4 or rank_slab or aspect" tests/test_gpu_multidevice.py::test_c3_strong_decomposition_exchange_accounting -x -v -s --timeout 880 --timeout-method thread > $O/tests.log 2>&1 || exit 4
