# GPU box: single-GPU RHS at the per-rank size of the 8-way run (1.25M elements) and at 2.5M / 5M, and the
# OMP-semantics bench at syn-10M.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g24
mkdir -p $O
A="--no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0 --steps 100 --warmup 5"
for n in 1250000 2500000 5000000; do
  timeout -k 10 300 python bench.py $A --n-ele $n > $O/rhs_$n.json 2> $O/rhs_$n.err
done
timeout -k 10 300 python bench.py $A --mode omp > $O/rhs_omp.json 2> $O/rhs_omp.err
echo done
