#!/bin/bash
# GPU box: per-phase attribution of the element kernel.  For the production library and each
# timing-only ablation build (tools/ablib.sh NAME -DSHUD_EABL=k / -DSHUD_ABL=k; results are wrong by design):
#   one rocprofv3 --pmc pass (SQ_WAVES, SQ_INSTS_VALU/SALU/VMEM/LDS, TRANS_F64, GRBM_GUI_ACTIVE) over the RHS-only bench,
#   then all libraries timed side by side in one process (tools/ab_variants.py, interleaved rounds).
#   usage: bash tools/ele_phase_attr.sh OUTDIR LIB1,LIB2,...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; libs=$2
mkdir -p "$O"
B="python3 bench.py --steps 5 --warmup 1 --settle 20 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
vs="pk"
for n in prod ${libs//,/ }; do
  if [ $n = prod ]; then L=""; else L=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so; vs="$vs,lib:$n"; fi
  SHUD_RHS_LIB=$L timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/sq_$n" -o run -- $B > "$O/sq_$n.log" 2>&1
  echo "[$(date +%T)] pmc $n done"
done
timeout -k 10 600 python3 tools/ab_variants.py --variants $vs --rounds 5 --reps 20 > "$O/abl.log" 2>&1
python3 tools/ele_phase_summary.py "$O" prod ${libs//,/ } > "$O/phase_attr.txt"
echo done
