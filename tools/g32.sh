# GPU box: the bench's N>1 code path on one rank (shared_partition + partitioned handle + RCCL comm), the driver
# command, smoke().
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g32
mkdir -p $O
timeout -k 10 300 python bench.py --partition-1 --steps 20 --warmup 5 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0 > $O/bench_p1.json 2> $O/bench_p1.err
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
echo done
