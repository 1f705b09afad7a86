# GPU box: integrator vector kernels, 4-deep load batches (default) vs one (SHUD_ODE_UNROLL=1): parity tests,
# syn-10M integrator A/B (bench's ode_timing), per-kernel stats of both, syn-1M shud_gpu day loop of both.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g17
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_ode.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread > $O/pytest_ode.log 2>&1
B="python3 bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-et --no-many-class --no-host-vectors --e2e-ele 0"
for k in 1 2; do
  for u in 1 4; do
    SHUD_ODE_UNROLL=$u timeout -k 10 300 $B > $O/ode_u${u}_$k.json 2> $O/ode_u${u}_$k.err
  done
done
for u in 1 4; do
  SHUD_ODE_UNROLL=$u timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_u$u -o run -- $B > $O/kt_u$u.log 2>&1
done
D=/tmp/shud_e2e_1M
timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0, 'shud-up_amd')
from shud_rhs import synth
synth.write_project('$D', 'syn', 1000000, days=1)
print('project written', flush=True)"
for u in 1 4 1 4; do
  SHUD_ODE_UNROLL=$u timeout -k 10 300 shud-up_amd/shud_gpu -q -o $D/out -C $D $D syn >> $O/e2e_u$u.log 2>&1
done
echo done
