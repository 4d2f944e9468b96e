#!/bin/bash
# round 6 (s): the forward y pass after a halo exchange's wait as ONE launch over the planes
# [0, cz) and [nz - cz, Mz) instead of two (SPIMDECON_YMERGE=0: two).  The two small launches
# (12 and 36 planes at 540: 204 and 612 tiles for 512 slots) each ran a partial round.
# Prediction: ~10 us per forward pass with neighbours, 12 per iteration: c3x8 / 2-3 local
# slab runs +0.5..1 %; bit-identical psi
export TMPDIR=/tmp
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_multidevice.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; tail -1 $O/tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python3 - > $O/bits.log 2>&1 <<'PY' || { echo "bits failed"; tail $O/bits.log; exit 1; }
import os, subprocess, sys, json, hashlib
code = r'''
import sys, hashlib, numpy as np
sys.path.insert(0, ".")
from spim_registration_amd import synthetic
from spim_registration_amd.decon import Session, PSFTYPE
imgs, ws, ks, _ = synthetic.make_views((60, 20, 248), 2, config_id=11, ksize=(9, 7, 9), weights="blend", partial=True, bead_density=1.0 / 6 ** 3)
with Session((248, 20, 60), local_slabs=3) as s:
    for i, w, k in zip(imgs, ws, ks): s.add_view(i, w, k)
    s.init(PSFTYPE.OPTIMIZATION_I); s.init_psi(); st = s.run(3, 0.006); psi = s.get_psi()
print(hashlib.sha256(psi.tobytes() + st.tobytes()).hexdigest())
'''
out = []
for ym in ("0", "1"):
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=dict(os.environ, SPIMDECON_YMERGE=ym))
    assert r.returncode == 0, r.stderr[-2000:]
    out.append(r.stdout.strip().splitlines()[-1])
print("ymerge0", out[0]); print("ymerge1", out[1]); print("bit-identical", out[0] == out[1])
assert out[0] == out[1]
PY
tail -1 $O/bits.log
for k in 1 2; do
  for ym in 0 1; do
    SPIMDECON_YMERGE=$ym timeout -k 10 240 python3 bench.py --no-cpu-baseline --strong --local-slabs 8 --steps 4 --warmup 1 --no-default-mode --no-strong-line > $O/c3x8_${ym}_$k.json 2> $O/c3x8_${ym}_$k.err || { echo "c3x8 failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/c3x8_${ym}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('c3x8 ymerge=$ym $k value %.1f ms %.2f y %.3f' % (d['value'], d['ms_per_step'], k['y_pass']['avg_ms']))"
    SPIMDECON_YMERGE=$ym timeout -k 10 240 python3 bench.py --no-cpu-baseline --no-default-mode --no-strong-line --steps 6 --warmup 1 --shape 512 512 1536 --local-slabs 3 --slab-axis z > $O/w3_${ym}_$k.json 2> $O/w3_${ym}_$k.err || { echo "w3 failed"; exit 1; }
    python3 -c "
import json; d=json.loads(open('$O/w3_${ym}_$k.json').read().strip().splitlines()[-1]); k=d['kernel_ms']
print('w3 ymerge=$ym $k value %.1f ms %.2f y %.3f' % (d['value'], d['ms_per_step'], k['y_pass']['avg_ms']))"
  done
done
echo done-r6s
