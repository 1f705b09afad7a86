#!/bin/bash
# GPU box: interleaved A/B of library variants at several mesh sizes (tools/ab_variants.py), optional GPU suite first.
# usage: bash tools/ab_sizes.sh OUTDIR VARIANTS ROUNDS SIZE [SIZE...]   (env SUITE=1: run pytest -m gpu first)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; V=$2; R=$3; shift 3
mkdir -p $O
if [ "${SUITE:-0}" = 1 ]; then
  timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1
fi
for n in "$@"; do
  timeout -k 10 ${ABT:-400} python tools/ab_variants.py --n-ele $n --variants $V --rounds $R --reps 50 ${ABX:-} > $O/abv_$n${ABS:-}.log 2>&1
done
echo done
