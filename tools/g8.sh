set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g8
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g8/pytest_gpu.log 2>&1
timeout -k 10 600 bash tools/profile_e2e.sh 1000000 1 > gpurun_out/g8/e2e.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline --e2e-ele 0 > gpurun_out/g8/bench.json 2> gpurun_out/g8/bench.err
echo done
