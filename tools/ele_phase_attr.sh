#!/bin/bash
# GPU box: per-phase attribution of the element kernel.  For the production library and each
# timing-only ablation build (tools/ablib.sh NAME -DSHUD_EABL=k / -DSHUD_ABL=k; results are wrong by design, so the
# bench's physics-error exit is expected and ignored):
#   one rocprofv3 --pmc pass (SQ_WAVES, SQ_INSTS_VALU/SALU/VMEM/LDS, TRANS_F64, GRBM_GUI_ACTIVE) over the RHS-only bench
#   per library in PMC_LIBS, then the libraries of TIME_LIBS timed side by side in one process (tools/ab_variants.py,
#   interleaved rounds).  Summary: python tools/ele_phase_summary.py OUTDIR prod LIB...
#   usage: bash tools/ele_phase_attr.sh OUTDIR PMC_LIBS TIME_LIBS     (comma lists; "prod" = the production library)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; plibs=$2; tlibs=$3
mkdir -p "$O"
B="python3 bench.py --steps 5 --warmup 1 --settle 20 --no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
for n in ${plibs//,/ }; do
  if [ $n = prod ]; then L=""; else L=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so; fi
  SHUD_RHS_LIB=$L timeout -k 10 240 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU_TRANS_F64 SQ_WAVE_CYCLES GRBM_GUI_ACTIVE --output-format csv -d "$O/sq_$n" -o run -- $B > "$O/sq_$n.log" 2>&1
  rc=$?
  echo "[$(date +%T)] pmc $n exit $rc"
  # a time limit, a crash or an abort ends the call (exit 3 = the ablation's expected physics-error flag)
  if [ $rc -ne 0 ] && [ $rc -ne 3 ]; then exit $rc; fi
done
if [ -n "$tlibs" ]; then
  vs="pk"
  for n in ${tlibs//,/ }; do [ $n = prod ] || vs="$vs,lib:$n"; done
  timeout -k 10 600 python3 tools/ab_variants.py --variants $vs --rounds 5 --reps 20 > "$O/abl.log" 2>&1 || exit $?
fi
echo done
