set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g7
timeout -k 10 300 python tools/traj_day.py gpurun_out/g7/traj_ccw_day.json > gpurun_out/g7/traj.log 2>&1
NE=1000000
D=/tmp/shud_e2e_$NE
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'shud-up_amd')
from shud_rhs import synth
synth.write_project('$D', 'syn', $NE, days=1)"
timeout -k 10 300 shud-up_amd/shud_gpu -q -o $D/out -C $D $D syn > gpurun_out/g7/e2e.log 2>&1
echo done
