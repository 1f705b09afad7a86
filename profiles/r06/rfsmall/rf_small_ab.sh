set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/r06/rfsmall
for n in 1000000 1250000; do
  timeout -k 10 300 python tools/ab_variants.py --n-ele $n --variants lib:rfold+SHUD_RHS_RFOLD=0,lib:rfold+SHUD_RHS_RFOLD=1 --rounds 9 --reps 50 > gpurun_out/r06/rfsmall/abv_$n.log 2>&1
done
echo done
