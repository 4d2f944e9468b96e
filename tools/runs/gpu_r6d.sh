#!/bin/bash
# round 6 (d): QPF on the fp16 2100 quotient wave tiles now default (r6c: quotient 1.95 -> 1.77 ms);
# A/B wp: the fp16 update wave tiles load psi + weights with the spectra (240 VGPRs, 8 waves
# per CU instead of 9); predicted update 2.84 -> ~2.6 ms if the exposed voxel round trips
# dominate, else neutral (one wave per CU fewer)
export TMPDIR=/tmp
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py tests/test_gpu_scale.py -x -q -k "x_tiles_2100 or c5_rank_slab" --timeout 500 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -2 $O/tests.log; [ $rc = 0 ] || exit 1
SPIMDECON_LIB=exp/libspimdecon_wp.so timeout -k 10 600 python -u -m pytest tests/test_gpu_rl.py -x -q -k "x_tiles_2100" --timeout 500 --timeout-method thread > $O/tests_wp.log 2>&1; rc=$?; tail -2 $O/tests_wp.log; [ $rc = 0 ] || exit 1
ext() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernel_ms") or {}
print(sys.argv[2], "value %.1f" % d["value"], " ".join("%s %.3f" % (c, k[c]["avg_ms"]) for c in ("x_quotient", "x_update", "y_pass", "z_convolve") if c in k))
PY
}
for k in 1 2 3; do
  for v in main wp; do
    L=spim_registration_amd/libspimdecon.so; [ $v = main ] || L=exp/libspimdecon_$v.so
    SPIMDECON_LIB=$L timeout -k 10 240 python3 bench.py --no-cpu-baseline --c5-rank --steps 4 --warmup 1 > $O/c5_${v}_$k.json 2> $O/c5_${v}_$k.err || { echo "c5 $v failed"; tail $O/c5_${v}_$k.err; exit 1; }
    ext $O/c5_${v}_$k.json "c5 $v $k"
  done
done
echo done-r6d
