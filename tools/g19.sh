# GPU box: split river path (junction kernel beside the element kernel) vs fused (SHUD_RIV_SPLIT=0): full GPU
# suite, RHS-only bench A/B, kernel trace of the split path.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g19
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
A="--no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
for k in 1 2; do
  for sp in 0 1; do
    SHUD_RIV_SPLIT=$sp timeout -k 10 300 python3 bench.py $A --steps 100 --warmup 5 > $O/rhs_s${sp}_$k.json 2> $O/rhs_s${sp}_$k.err
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $A --steps 20 --warmup 5 > $O/kt.log 2>&1
echo done
