#!/bin/bash
# round 6 (n): C4 pipeline stage times, twice (r6j showed detect 68-70 ms on timepoints 0-1
# against 38-40 ms on 2-3 and in round 5: box noise or the new PSF workspace release?)
export TMPDIR=/tmp
O=gpurun_out/r6n
mkdir -p $O
for k in 1 2; do
  timeout -k 10 400 python3 tools/c4_pipeline.py > $O/c4_$k.log 2>&1 || { echo "c4 failed"; tail -5 $O/c4_$k.log; exit 1; }
  python3 - $O/c4_$k.log <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
for t in d["timepoints"]:
    s = t["stage_ms"]
    print(t["t"], t["s"], {k: s[k] for k in ("detect", "correspondences", "prepare_inputs", "extract_psf", "rl_setup", "rl_iterations")})
print("total", d["total_s"], "per timepoint", d["s_per_timepoint"])
PY
done
echo done-r6n
