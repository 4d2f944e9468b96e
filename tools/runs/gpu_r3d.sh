#!/bin/bash
# round-3: DoG bit-exactness + A/B (prefetch depth, chunk), z-pass buffers, large-geometry tests
export TMPDIR=/tmp
O=gpurun_out/r3d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_dog.py tests/test_gpu_configs.py::test_c4_dog_768_matches_oracle_on_crops -x -q --timeout 250 --timeout-method thread > $O/dog_tests.log 2>&1 || exit 1
tools/dog_ab.sh $O/dogab "SPIMDECON_DOG_PD=8" "SPIMDECON_DOG_PD=3" "SPIMDECON_DOG_PD=8 SPIMDECON_DOG_ZCHUNK=128" "SPIMDECON_DOG_PD=8 SPIMDECON_DOG_XCD=0" || exit 2
for nb in 3 2; do
  SPIMDECON_ZNB=$nb timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-strong-line --no-default-mode > $O/bench_znb$nb.log 2>&1 || exit 3
done
timeout -k 10 800 python -u -m pytest tests/test_gpu_scale.py -k "c5_full or c4 or rank_slab or aspect" -x -v -s --timeout 780 --timeout-method thread > $O/tests.log 2>&1 || exit 4
