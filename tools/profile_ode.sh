#!/bin/bash
# GPU box: integrator parity tests, then a kernel trace of the bench (ET prelude + device integrator timing)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_ode.py tests/test_gpu_out.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_ode.log 2>&1
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ode -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --profile-reps 2 > gpurun_out/bench_ode.json 2> gpurun_out/bench_ode.err
echo done
