#!/bin/bash
# GPU box: edge sharing on vs off (same library) across mesh sizes and for the 8-way rank.
# usage: bash tools/share_sweep.sh OUTDIR
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1
mkdir -p $O
for n in 1000000 2500000 5000000; do
  timeout -k 10 400 python tools/ab_variants.py --n-ele $n --variants pk,pk+SHUD_RHS_SHARE=0 --rounds 5 --reps 50 > $O/abv_$n.log 2>&1
done
timeout -k 10 300 python tools/rank_timing.py 8 > $O/rank8_share.json 2> $O/rank8_share.err
SHUD_RHS_SHARE=0 timeout -k 10 300 python tools/rank_timing.py 8 > $O/rank8_noshare.json 2> $O/rank8_noshare.err
echo done
