#!/bin/bash
# Per-class engine times of the BASELINE geometries on one GPU (gpurun): OUT/<name>.json and
# OUT/engine_classes.json {name: {value, ms_per_step, pointwise, kernel_ms, config}}
# usage: tools/engine_classes.sh OUT
set -o pipefail
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
declare -A CFG=(
  [headline]="--steps 10 --no-strong-line"
  [c3]="--strong --steps 4 --warmup 1 --no-default-mode --no-strong-line"
  [c3x8]="--strong --local-slabs 8 --steps 4 --warmup 1 --no-default-mode --no-strong-line"
  [c4]="--shape 768 768 768 --views 8 --psftype OPTIMIZATION_I --lam 0.006 --steps 4 --warmup 1 --no-default-mode --no-strong-line"
  [c5]="--c5-rank --steps 4 --warmup 1"
  [c3rank]="--c3-rank --steps 6 --warmup 2"
)
for n in ${CLASSES:-headline c3 c3x8 c3rank c4 c5}; do
  timeout -k 10 300 python3 bench.py --no-cpu-baseline --no-legacy-line ${CFG[$n]} > $OUT/$n.log 2>&1 || { echo "$n failed"; tail -5 $OUT/$n.log; exit 1; }
  tail -1 $OUT/$n.log > $OUT/$n.json
  python3 - $OUT/$n.json $n <<'PY'
import json, sys
d = json.load(open(sys.argv[1]))
k = d.get("kernel_ms") or {}
pw = d.get("pointwise") or {}
dm = d.get("default_mode") or {}
print(sys.argv[2], "value %.1f ms %.3f" % (d["value"], d["ms_per_step"]),
      "pointwise %.3f" % pw.get("frac", float("nan")), " ".join("%s %.3f" % (c, k[c]["avg_ms"]) for c in ("x_quotient", "x_update", "y_pass", "z_convolve") if c in k),
      ("default %.1f pointwise %.3f" % (dm["value"], (dm.get("pointwise") or {}).get("frac", float("nan")))) if dm else "")
PY
done
python3 - $OUT <<'PY'
import json, os, sys
out = {}
for n in ("headline", "c3", "c3x8", "c3rank", "c4", "c5"):
    if not os.path.exists(os.path.join(sys.argv[1], n + ".json")):
        continue
    d = json.load(open(os.path.join(sys.argv[1], n + ".json")))
    out[n] = {k: d.get(k) for k in ("value", "ms_per_step", "pointwise", "kernel_ms", "roofline", "config", "default_mode")}
json.dump(out, open(os.path.join(sys.argv[1], "engine_classes.json"), "w"), indent=1)
PY
