# GPU box: full GPU suite, then the round profile (tools/profile_round.sh).
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/g14
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/g14/pytest_gpu.log 2>&1
timeout -k 10 1200 bash tools/profile_round.sh > gpurun_out/g14/profile_round.log 2>&1
echo done
