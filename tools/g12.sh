set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g12
timeout -k 10 600 python -u -m pytest tests/test_gpu_ode.py tests/test_gpu_host.py tests/test_gpu_out.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g12/pytest.log 2>&1
timeout -k 10 600 bash tools/profile_e2e.sh 1000000 1 > gpurun_out/g12/e2e.log 2>&1
timeout -k 10 400 python bench.py --no-cpu-baseline --no-many-class --no-host-vectors --steps 20 > gpurun_out/g12/bench.json 2> gpurun_out/g12/bench.err
echo done
