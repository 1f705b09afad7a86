#!/bin/bash
# GPU box: parity suite, A/B libs (tools/ablib.sh names given as args), bench line.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1
if [ $# -gt 0 ]; then timeout -k 10 600 bash tools/ab_libs.sh "$@" > gpurun_out/ab_summary.log 2>&1; fi
timeout -k 10 400 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
echo done
