# GPU box: four-lane river kernel for small reach counts — GPU suite, per-rank times with / without it,
# syn-1M RHS with / without it.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g29
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
A="--no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0 --steps 100 --warmup 5 --n-ele 1000000"
for q in 0 1 0 1; do
  SHUD_RIV_QUAD=$q timeout -k 10 300 python bench.py $A >> $O/rhs1m_q$q.jsonl 2>> $O/rhs1m.err
done
timeout -k 10 600 python -u tools/rank_timing.py 8 4 2 > $O/rt_quad.json 2> $O/rt_quad.err
SHUD_RIV_QUAD=0 timeout -k 10 600 python -u tools/rank_timing.py 8 4 2 > $O/rt_single.json 2> $O/rt_single.err
echo done
