# GPU box: boundary elements concurrent with the interior elements (side stream) vs serial, per-rank at 8 ranks;
# partition parity tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g26
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_host.py -x -q --timeout 300 --timeout-method thread > $O/pytest_part.log 2>&1
timeout -k 10 600 python -u tools/rank_timing.py 8 4 > $O/rt_conc.json 2> $O/rt_conc.err
SHUD_RHS_BND_CONCURRENT=0 timeout -k 10 600 python -u tools/rank_timing.py 8 4 > $O/rt_serial.json 2> $O/rt_serial.err
timeout -k 10 300 python bench.py --partition-1 --steps 20 --warmup 5 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0 > $O/bench_p1.json 2> $O/bench_p1.err
echo done
