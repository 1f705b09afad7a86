# GPU box: full GPU suite (edge meshes, ragged partitions) and the driver bench command.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g16
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g16/pytest_gpu.log 2>&1
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/g16/bench.json 2> gpurun_out/g16/bench.err
echo done
