#!/bin/bash
# GPU box: end-to-end shud_gpu (C++ host, device ET prelude + RHS + integrator + outputs) on a synthetic project,
# plain and under a rocprofv3 kernel trace (per-kernel GPU time of the whole SHUD() loop).
# usage: bash tools/profile_e2e.sh [NE] [DAYS]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
NE=${1:-1000000}
DAYS=${2:-1}
O=gpurun_out/e2e
mkdir -p $O
D=/tmp/shud_e2e_$NE
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'shud-up_amd')
from shud_rhs import synth
synth.write_project('$D', 'syn', $NE, days=$DAYS)
print('project written', flush=True)"
timeout -k 10 300 shud-up_amd/shud_gpu -q -o $D/out -C $D $D syn > $O/e2e_$NE.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_$NE -o run -- shud-up_amd/shud_gpu -q -o $D/out2 -C $D $D syn > $O/e2e_kt_$NE.log 2>&1
tail -2 $O/e2e_$NE.log
echo done
