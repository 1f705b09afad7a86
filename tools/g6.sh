set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g6
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 240 --timeout-method thread > gpurun_out/g6/pytest_gpu.log 2>&1
SHUD_RHS_LIB=$PWD/shud-up_amd/build/ab/libshud_rhs_cdiv.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 240 --timeout-method thread > gpurun_out/g6/pytest_cdiv.log 2>&1 || echo "cdiv parity failed" >> gpurun_out/g6/pytest_cdiv.log
timeout -k 10 600 bash tools/ab_libs.sh cdiv > gpurun_out/g6/ab.log 2>&1
timeout -k 10 300 python tools/riv_abl.py > gpurun_out/g6/rivabl.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/g6/fetch -o run -- python3 tools/riv_abl.py > gpurun_out/g6/fetch.log 2>&1
timeout -k 10 600 bash tools/profile_e2e.sh 1000000 1 > gpurun_out/g6/e2e.log 2>&1
echo done
