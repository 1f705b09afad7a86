# GPU box: full GPU suite, the driver's bench command, the N>1 path on one rank, per-rank times of the N>1
# decomposition (tools/rank_timing.py).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g23
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python bench.py --partition-1 --steps 20 --warmup 5 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0 > $O/bench_p1.json 2> $O/bench_p1.err
timeout -k 10 600 python -u tools/rank_timing.py 2 4 8 > $O/rank_timing.json 2> $O/rank_timing.err
echo done
