# GPU box: randomized GPU property tests (hypothesis), then the integrator tests again.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g21
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py -x -v --timeout 300 --timeout-method thread > $O/pytest_props.log 2>&1
echo done
