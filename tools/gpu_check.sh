#!/bin/bash
# GPU box: parity suite + stream sweep + a short bench line (no CPU baseline / ET / integrator / e2e)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/check
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > $O/pytest_gpu.log 2>&1
if [ -x tools/stream_sweep ]; then timeout -k 10 120 tools/stream_sweep > $O/stream_sweep.log 2>&1; fi
timeout -k 10 400 python bench.py --no-cpu-baseline --no-et --no-ode --e2e-ele 0 $BENCH_ARGS > $O/bench.json 2> $O/bench.err
echo done
