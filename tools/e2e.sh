#!/bin/bash
# GPU box: end-to-end SHUD() on the device through the C++ host (shud_gpu) on a synthetic
# project written in SHUD text format: NE elements, DAYS simulated days, hourly forcing, hourly outputs.
# usage: bash tools/e2e.sh [NE] [DAYS]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
NE=${1:-1000000}
DAYS=${2:-1}
D=/tmp/shud_e2e_$NE
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'shud-up_amd')
from shud_rhs import synth
synth.write_project('$D', 'syn', $NE, days=$DAYS)
print('project written', flush=True)"
timeout -k 10 600 shud-up_amd/shud_gpu -o $D/out -C $D $D syn > gpurun_out/e2e_$NE.log 2>&1
tail -3 gpurun_out/e2e_$NE.log
ls $D/out | head -3 >> gpurun_out/e2e_$NE.log
