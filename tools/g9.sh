set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g9
timeout -k 10 400 python -u -m pytest tests/test_gpu_host.py tests/test_gpu_out.py -x -q --timeout 240 --timeout-method thread > gpurun_out/g9/pytest_host.log 2>&1
timeout -k 10 600 bash tools/profile_e2e.sh 1000000 1 > gpurun_out/g9/e2e.log 2>&1
echo done
