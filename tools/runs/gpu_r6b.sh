#!/bin/bash
# round 6 (b): wave x tiles (one wave per block, no block barrier between waves) A/B.
# Prediction (r6a PMC: 2100 tiles one 8-wave block per CU, VALU ~45 % busy, load / store /
# image-load phases serialised behind block barriers): C5 quotient 2.33 -> ~1.9 ms, update
# 3.01 -> ~2.6 ms if the resident waves overlap their HBM phases; 1050 likewise -5..-15 %.
export TMPDIR=/tmp
O=gpurun_out/r6b
mkdir -p $O
ext() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d["kernel_ms"] if "kernel_ms" in d else {}
print(sys.argv[2], "value %.1f" % d["value"], " ".join("%s %.3f" % (c, k[c]["avg_ms"]) for c in ("x_quotient", "x_update", "y_pass", "z_convolve") if c in k))
PY
}
for k in 1 2; do
  for v in main w2100 w2100w3; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 200 python3 bench.py --c5-rank --steps 4 --warmup 1 --no-cpu-baseline > $O/c5_${v}_$k.json 2> $O/c5_${v}_$k.err || { echo "c5 $v failed"; tail $O/c5_${v}_$k.err; exit 1; }
    ext $O/c5_${v}_$k.json "c5 $v $k"
  done
  for v in main w1050; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 200 python3 bench.py --strong --steps 3 --warmup 1 --no-cpu-baseline --no-default-mode --no-strong-line > $O/c3_${v}_$k.json 2> $O/c3_${v}_$k.err || { echo "c3 $v failed"; tail $O/c3_${v}_$k.err; exit 1; }
    ext $O/c3_${v}_$k.json "c3 $v $k"
  done
done
SPIMDECON_LIB=exp/libspimdecon_w1050.so timeout -k 10 400 python -u -m pytest tests/test_gpu_rl.py -x -q -k "tikhonov_update_tiles" --timeout 300 --timeout-method thread > $O/tests_w1050.log 2>&1; echo "w1050 tests rc=$?"; tail -2 $O/tests_w1050.log
echo done-r6b
