#!/bin/bash
# river-kernel ablations.  Here (build): bash tools/riv_abl.sh build   -> build/ab/libshud_rhs_rabl{1,2,4,7}.so
# GPU box: bash tools/riv_abl.sh [outdir]  -> times + FETCH/WRITE passes per library
set -e
if [ "$1" = build ]; then
  for k in 1 2 4 7; do bash "$(dirname "$0")/ablib.sh" rabl$k -DSHUD_RIV_ABL=$k; done
  exit 0
fi
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=${1:-gpurun_out/rivabl}
mkdir -p $O
for k in prod 1 2 4 7; do
  if [ $k = prod ]; then L=""; else L=$PWD/shud-up_amd/build/ab/libshud_rhs_rabl$k.so; fi
  SHUD_RHS_LIB=$L timeout -k 10 300 python tools/riv_abl.py 10000000 abl$k >> $O/times.log 2>&1
  SHUD_RHS_LIB=$L timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch$k -o run -- python3 tools/riv_abl.py 10000000 abl$k > $O/fetch$k.log 2>&1
  SHUD_RHS_LIB=$L timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $O/write$k -o run -- python3 tools/riv_abl.py 10000000 abl$k > $O/write$k.log 2>&1
done
echo done
