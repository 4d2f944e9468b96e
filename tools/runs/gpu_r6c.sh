#!/bin/bash
# round 6 (c): wave x tiles at 2100 now the default -- its tests; then A/B of
#  wu  (update wave tiles with the two-slot voxel pipeline; predicted C5 update 2.84 -> ~2.65 ms),
#  wq  (fp16 quotient wave tiles load the image rows before the inverse transform, 170 VGPRs,
#       8 waves per CU as the LDS allows 9; predicted quotient 1.95 -> ~1.85 ms),
#  w540 / w800 (wave tiles of 2 row pairs at 540 / 800: 540 blocks already overlap 4 per CU,
#       predicted within +-2 %; 800 at 3 blocks per CU, predicted C4-shape RL -2..+5 %)
export TMPDIR=/tmp
O=gpurun_out/r6c
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_scale.py -x -q -k "x_tiles_2100 or c5_rank_slab or c5_decomposition" --timeout 600 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -3 $O/tests.log; [ $rc = 0 ] || exit 1
ext() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernel_ms") or {}
dm = d.get("default_mode") or {}
print(sys.argv[2], "value %.1f" % d["value"], " ".join("%s %.3f" % (c, k[c]["avg_ms"]) for c in ("x_quotient", "x_update", "y_pass", "z_convolve") if c in k),
      ("default %.1f" % dm["value"]) if dm else "")
PY
}
run() {  # tag variant args...
  local tag=$1 v=$2; shift 2
  L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
  SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline "$@" > $O/${tag}_$v.json 2> $O/${tag}_$v.err || { echo "$tag $v failed"; tail $O/${tag}_$v.err; exit 1; }
  ext $O/${tag}_$v.json "$tag $v"
}
for k in 1 2; do
  for v in main wu wq wuq; do run c5_$k $v --c5-rank --steps 4 --warmup 1; done
  for v in main w540; do run h_$k $v --steps 10 --no-strong-line; done
  for v in main w800; do run c4_$k $v --shape 768 768 768 --views 8 --psftype OPTIMIZATION_I --lam 0.006 --steps 4 --no-strong-line --no-default-mode; done
done
echo done-r6c
