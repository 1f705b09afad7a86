#!/bin/bash
# GPU box: kernel trace of the bench with the device integrator timing (per-kernel share of an integrator step)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_ode -o run -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-et --profile-reps 2 > gpurun_out/bench_ode.json 2> gpurun_out/bench_ode.err
echo done
