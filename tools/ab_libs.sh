#!/bin/bash
# GPU box: time the production lib and each A/B lib built by tools/ablib.sh (one process per lib).
#   tools/ab_libs.sh name1 name2 ...   -> gpurun_out/ab_<name>.log
set -e
mkdir -p gpurun_out
timeout -k 10 300 python tools/ab_variants.py --variants pk --rounds 5 > gpurun_out/ab_prod.log 2>&1
for n in "$@"; do
  SHUD_RHS_LIB=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so timeout -k 10 300 python tools/ab_variants.py --variants pk --rounds 5 > gpurun_out/ab_$n.log 2>&1
done
for f in prod "$@"; do echo "$f $(tail -n 1 gpurun_out/ab_$f.log)"; done
