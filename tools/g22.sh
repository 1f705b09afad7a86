# GPU box: lakes in partitioned handles + randomized GPU property tests.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g22
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_partition.py tests/test_gpu_parity.py -k lake -x -v --timeout 300 --timeout-method thread > $O/pytest_lakes.log 2>&1
timeout -k 10 600 python -u -m pytest tests/test_gpu_properties.py -x -v --timeout 300 --timeout-method thread > $O/pytest_props.log 2>&1
echo done
