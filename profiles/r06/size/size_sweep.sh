#!/bin/bash
# GPU box: the packed RHS across mesh sizes (per-element cost vs size) + SQ counters at the 8-way rank's size.
# usage: bash tools/size_sweep.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/size}
mkdir -p $O
for n in 1250000 2500000 5000000 10000000; do
  timeout -k 10 300 python tools/ab_variants.py --n-ele $n --variants pk --rounds 3 --reps 50 > $O/abv_$n.log 2>&1
done
B="python3 bench.py --steps 5 --warmup 1 --n-ele 1250000 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o run -- $B > $O/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.log 2>&1
python3 tools/sq_summary.py $O > $O/sq_summary.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/kt -o run -- $B > $O/kt.log 2>&1
echo done
