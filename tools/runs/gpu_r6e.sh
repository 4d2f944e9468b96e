#!/bin/bash
# round 6 (e): the whole -m gpu suite at HEAD (wave x tiles at 2100, RCCL watchdog / rank
# check / one-rank communicator, PSF workspace release, JNA child, concurrent boundary
# launches), the smoke; then A/B of the concurrent boundary launches on C3's 8-rank slabs
# emulated on one GPU (bench --strong --local-slabs 8).  Prediction: the boundary launch's
# tail and the launch gap hidden, 12 split passes per iteration x ~15 us = ~0.2 ms of 8.3 ms
# per slab: c3x8 +1..3 %
export TMPDIR=/tmp
O=gpurun_out/r6e
mkdir -p $O
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 600 --timeout-method thread --durations 15 > $O/tests.log 2>&1; rc=$?; tail -22 $O/tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; tail -2 $O/smoke.log; [ $rc = 0 ] || exit 1
ext() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
k = d.get("kernel_ms") or {}
print(sys.argv[2], "value %.1f ms %.2f" % (d["value"], d["ms_per_step"]), " ".join("%s %.3f" % (c, k[c]["avg_ms"]) for c in ("x_quotient", "x_update", "y_pass", "z_convolve", "halo_exchange", "exchange_window") if c in k))
PY
}
for k in 1 2; do
  for cb in 0 1; do
    SPIMDECON_CBND=$cb timeout -k 10 240 python3 bench.py --no-cpu-baseline --strong --local-slabs 8 --steps 4 --warmup 1 --no-default-mode --no-strong-line > $O/c3x8_cb${cb}_$k.json 2> $O/c3x8_cb${cb}_$k.err || { echo "c3x8 cb$cb failed"; tail $O/c3x8_cb${cb}_$k.err; exit 1; }
    ext $O/c3x8_cb${cb}_$k.json "c3x8 cbnd=$cb $k"
  done
done
echo done-r6e
