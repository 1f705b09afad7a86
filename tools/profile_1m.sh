#!/bin/bash
# GPU box: BASELINE configs[3] — syn-1M on one GPU: bench line, kernel trace, HBM PMC passes (separate runs)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/syn1M}
mkdir -p "$O"
A="--n-ele 1000000 --no-et --no-ode --e2e-ele 0"
timeout -k 10 300 python bench.py $A --steps 200 --warmup 10 > "$O/bench.json" 2> "$O"/bench.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O"/kt -o run -- python3 bench.py $A --steps 50 --warmup 5 --no-cpu-baseline > "$O"/bench_kt.json 2> "$O"/bench_kt.err
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O"/fetch -o run -- python3 bench.py $A --steps 5 --warmup 1 --no-cpu-baseline --profile-reps 2 > "$O"/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O"/write -o run -- python3 bench.py $A --steps 5 --warmup 1 --no-cpu-baseline --profile-reps 2 > "$O"/write.log 2>&1
echo done
