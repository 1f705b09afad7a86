#!/bin/bash
# GPU box: bench line + rocprofv3 kernel trace of the SAME bench command (its HIP-event kernel times and the
# trace's averages must agree) + HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs) -> pmc_summary
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/prof
mkdir -p $O
A="--no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- python3 bench.py $A --steps 100 --warmup 5 > $O/bench_kt.json 2> $O/bench_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py $A --steps 5 --warmup 1 > $O/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/pmc_write -o run -- python3 bench.py $A --steps 5 --warmup 1 > $O/pmc_write.log 2>&1
python tools/pmc_summary.py $O/pmc_fetch $O/pmc_write 10001406 $O/pmc_summary.json > /dev/null
echo done
