#!/bin/bash
# GPU box: SQ/GRBM counter passes over a short RHS-only bench run (kernel-trace only, no sys/runtime trace);
# one --pmc pass per block budget (<= 8 SQ, <= 2 GRBM counters per pass).  usage: bash tools/sq_counters.sh [outdir]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/prof}
mkdir -p $O
B="python3 bench.py --steps 5 --warmup 1 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d $O/sq1 -o run -- $B > $O/sq1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU_TRANS_F64 SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_ADD_F64 SQ_INSTS_VALU_MUL_F64 SQ_LDS_BANK_CONFLICT --output-format csv -d $O/sq2 -o run -- $B > $O/sq2.log 2>&1
python3 tools/sq_summary.py $O > $O/sq_summary.txt
echo done
