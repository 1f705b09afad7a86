#!/bin/bash
# GPU box: bench line + rocprofv3 kernel trace + HBM PMC passes (FETCH_SIZE and WRITE_SIZE in separate runs)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_kt -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-et --no-ode > gpurun_out/bench_kt.json 2> gpurun_out/bench_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-et --no-ode --profile-reps 2 > gpurun_out/pmc_fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-et --no-ode --profile-reps 2 > gpurun_out/pmc_write.log 2>&1
echo done
