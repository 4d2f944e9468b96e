#!/bin/bash
# round 4 (e): PMC passes of the fused y-z-y pass (opt-in) at the bench geometry
export TMPDIR=/tmp
O=gpurun_out/r4e
mkdir -p $O
export SPIMDECON_YZY=1
tools/pmc_engine.sh $O/pmc || exit 1
python3 tools/pmc_summary.py $O/pmc > $O/pmc.md || exit 2
