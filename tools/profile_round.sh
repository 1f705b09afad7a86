#!/bin/bash
# GPU box, end of a round: the driver's bench command, a rocprofv3 kernel trace of the same command (its HIP-event
# kernel times and the trace's averages must agree), the integrator's kernel trace, HBM PMC passes (FETCH_SIZE / WRITE_SIZE, separate runs) ->
# pmc_summary.json keyed to the kernel sources, SQ counters, the N>1 code path on one rank, the 1M end-to-end run.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
A="--no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $A --steps 20 --warmup 5 > $O/bench_kt.json 2> $O/bench_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py $A --steps 5 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py $A --steps 5 --warmup 1 > $O/pmc_write.log 2>&1
python3 tools/pmc_summary.py $O/pmc_fetch $O/pmc_write 10001406 $O/pmc_summary.json > /dev/null
timeout -k 10 300 bash tools/sq_counters.sh $O > /dev/null
timeout -k 10 300 python bench.py $A --partition-1 --steps 20 > $O/bench_partition1.json 2> $O/bench_partition1.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt_ode -o run -- python3 bench.py --no-cpu-baseline --no-et --no-many-class --no-host-vectors --e2e-ele 0 --steps 5 --warmup 1 > $O/bench_ode_kt.json 2> $O/bench_ode_kt.err
timeout -k 10 600 bash tools/profile_e2e.sh 1000000 1 > $O/e2e.log 2>&1
echo done
