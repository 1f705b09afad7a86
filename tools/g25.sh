# GPU box: where the partitioned per-rank overhead goes at 8 ranks (split launch, pack kernel), by ablation.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/g25
mkdir -p $O
timeout -k 10 600 python -u tools/rank_timing.py 8 > $O/rt_default.json 2> $O/rt_default.err
SHUD_RHS_NOSPLIT=1 timeout -k 10 600 python -u tools/rank_timing.py 8 > $O/rt_nosplit.json 2> $O/rt_nosplit.err
SHUD_RHS_NOPACK=1 timeout -k 10 600 python -u tools/rank_timing.py 8 > $O/rt_nopack.json 2> $O/rt_nopack.err
SHUD_RHS_NOSPLIT=1 SHUD_RHS_NOPACK=1 timeout -k 10 600 python -u tools/rank_timing.py 8 > $O/rt_none.json 2> $O/rt_none.err
echo done
