#!/bin/bash
# GPU box: one parameterised step runner for every gpurun call (replaces the per-call gNN.sh files).
#   bash tools/gpu_run.sh OUTDIR STEP [STEP ...]
# steps (each under its own timeout; the first failure ends the call):
#   suite        pytest -m gpu (full), log + durations        smoke     __graft_entry__.smoke()
#   bench        the driver's command: bench.py --gpus 1 --steps 20 --warmup 5
#   quick        RHS-only bench line (no CPU baseline / ET / integrator / e2e)
#   quickab:L1,L2  the RHS-only bench line for the production lib and each A/B lib, twice
#   abv:V1,V2    tools/ab_variants.py --variants V1,V2 (e.g. pk,pkR) on the production lib, 9 rounds
#   abl:L1,L2    tools/ab_variants.py, production + each A/B lib loaded side by side, interleaved per round
#   ab:L1,L2     tools/ab_variants.py (SoA reference + packed, bit-identity checked) on the production lib and each build/ab/libshud_rhs_<L>.so
#   odeab:L1,L2  integrator ms/step (bench.py integrator section) for the production lib and each A/B lib, twice
#   kt           rocprofv3 kernel trace of the RHS-only bench            pmc   FETCH_SIZE / WRITE_SIZE passes -> summary
#   calib        PMC calibration kernels (tools/calibrate_pmc)                tcc   L2 hit/miss of the RHS kernels
#   sq           SQ / GRBM counter passes (tools/sq_counters.sh)          ode   integrator kernel trace
#   part1        bench's N>1 code path on one rank                        rank  tools/rank_timing.py (2/4/8-way)
#   rankab:L1,L2 tools/rank_timing.py 8 for the production lib and each A/B lib   rankkt  its kernel trace (8-way)
#   rankjoin     8-way rank timing with / without the trailing comm-stream join (SHUD_RHS_FOLD_JOIN=1: join)
#   rankfold     8-way rank timing, boundary elements folded into the interior launch vs split (SHUD_RHS_FOLD=0)
#   syn1m        tools/profile_1m.sh (BASELINE configs[3]: bench line, kernel trace, PMC)   sizes  RHS lines at 1.25/2.5/5M + OMP
#   e2e          tools/profile_e2e.sh 1M, 1 day                          redbench  tools/ode_red_bench (reduction forms)
#   classes      tools/class_sweep.py (element kernel vs #parameter classes, LDS / L2 / SoA)
#   test:EXPR    pytest -m gpu -k EXPR                                    traj  tests/diag_traj_day.py (ccw one day)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=$1; shift
mkdir -p "$O"
A="--no-cpu-baseline --no-et --no-ode --no-many-class --no-host-vectors --e2e-ele 0"
for step in "$@"; do
  echo "[$(date +%T)] $step"
  case "$step" in
    suite) timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --durations=30 --timeout 240 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 ;;
    test:*) timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "${step#test:}" > "$O/pytest_sel.log" 2>&1 ;;
    abtest:*)                   # abtest:LIB:EXPR  -> pytest -m gpu -k EXPR against build/ab/libshud_rhs_LIB.so
      rest="${step#abtest:}"; lib="${rest%%:*}"; expr="${rest#*:}"
      SHUD_RHS_LIB=$PWD/shud-up_amd/build/ab/libshud_rhs_$lib.so timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread -k "$expr" > "$O/pytest_ab_$lib.log" 2>&1 ;;
    smoke) timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ;;
    bench) timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > "$O/bench.json" 2> "$O/bench.err" ;;
    quick) timeout -k 10 300 python bench.py $A --steps 20 --warmup 5 > "$O/quick.json" 2> "$O/quick.err" ;;
    quickab:*)                  # quickab:L1,L2 -> RHS-only bench line for the production lib and each A/B lib, 2 rounds
      libs="${step#quickab:}"
      for rep in 1 2; do
        for n in prod ${libs//,/ }; do
          if [ $n = prod ]; then L=""; else L=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so; fi
          SHUD_RHS_LIB=$L timeout -k 10 300 python bench.py $A --steps 40 --warmup 5 > "$O/quick_${n}_$rep.json" 2> "$O/quick_${n}_$rep.err"
          echo "$n rep$rep $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['ms_per_step'], d['roofline']['kernel_ms'])" "$O/quick_${n}_$rep.json")" >> "$O/quickab_summary.log"
        done
      done ;;
    abv:*)                      # abv:V1,V2 -> tools/ab_variants.py on the production lib with these variants, 9 rounds
      timeout -k 10 400 python tools/ab_variants.py --variants "${step#abv:}" --rounds 9 > "$O/abv.log" 2>&1
      tail -n 1 "$O/abv.log" > "$O/abv_summary.log" ;;
    abl:*)                      # abl:L1,L2 -> production packed kernel and each A/B lib interleaved in one process, 9 rounds
      libs="${step#abl:}"; vs="pk"
      for n in ${libs//,/ }; do vs="$vs,lib:$n"; done
      timeout -k 10 400 python tools/ab_variants.py --variants $vs --rounds 9 > "$O/abl.log" 2>&1
      tail -n 1 "$O/abl.log" > "$O/abl_summary.log" ;;
    ab:*)
      libs="${step#ab:}"
      timeout -k 10 300 python tools/ab_variants.py --variants soa,pk --rounds 5 > "$O/ab_prod.log" 2>&1
      for n in ${libs//,/ }; do
        SHUD_RHS_LIB=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so timeout -k 10 300 python tools/ab_variants.py --variants soa,pk --rounds 5 > "$O/ab_$n.log" 2>&1
      done
      for f in prod ${libs//,/ }; do echo "$f $(tail -n 1 "$O/ab_$f.log")"; done > "$O/ab_summary.log" ;;
    odeab:*)
      libs="${step#odeab:}"
      B="--no-cpu-baseline --no-et --no-many-class --no-host-vectors --e2e-ele 0 --steps 5 --warmup 1"
      for rep in 1 2; do
        for n in prod ${libs//,/ }; do
          if [ $n = prod ]; then L=""; else L=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so; fi
          SHUD_RHS_LIB=$L timeout -k 10 300 python bench.py $B > "$O/odeab_${n}_$rep.json" 2> "$O/odeab_${n}_$rep.err"
          echo "$n rep$rep $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['integrator']['ms_per_step'], d['integrator']['steps'])" "$O/odeab_${n}_$rep.json")" >> "$O/odeab_summary.log"
        done
      done ;;
    kt) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt" -o run -- python3 bench.py $A --steps 20 --warmup 5 > "$O/bench_kt.json" 2> "$O/bench_kt.err" ;;
    rankfold)                   # 8-way rank timing with the boundary launch folded (default) and split
      timeout -k 10 300 python tools/rank_timing.py 8 > "$O/rank8_fold.json" 2> "$O/rank8_fold.err"
      SHUD_RHS_FOLD=0 timeout -k 10 300 python tools/rank_timing.py 8 > "$O/rank8_split.json" 2> "$O/rank8_split.err" ;;
    rankjoin)                   # 8-way rank timing with / without the main stream's trailing join of the comm stream
      SHUD_RHS_FOLD_JOIN=1 timeout -k 10 300 python tools/rank_timing.py 8 > "$O/rank8_join.json" 2> "$O/rank8_join.err"
      timeout -k 10 300 python tools/rank_timing.py 8 > "$O/rank8_nojoin.json" 2> "$O/rank8_nojoin.err" ;;
    rankkt) timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d "$O/rankkt" -o run -- python3 tools/rank_timing.py 8 > "$O/rankkt.json" 2> "$O/rankkt.err" ;;
    pmc)
      timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/pmc_fetch" -o run -- python3 bench.py $A --steps 5 --warmup 1 > "$O/pmc_fetch.log" 2>&1
      timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/pmc_write" -o run -- python3 bench.py $A --steps 5 --warmup 1 > "$O/pmc_write.log" 2>&1
      python3 tools/pmc_summary.py "$O/pmc_fetch" "$O/pmc_write" 10001406 "$O/pmc_summary.json" 972842 5003338 > /dev/null ;;
    calib)                      # FETCH_SIZE / WRITE_SIZE of the known-byte kernels (tools/calibrate_pmc, built in-tree)
      timeout -k 10 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$O/calib_fetch" -o run -- ./tools/calibrate_pmc > "$O/calib_fetch.log" 2>&1
      timeout -k 10 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$O/calib_write" -o run -- ./tools/calibrate_pmc > "$O/calib_write.log" 2>&1
      python3 tools/pmc_counters.py "$O/calib_fetch" > "$O/calib_summary.txt"
      python3 tools/pmc_counters.py "$O/calib_write" >> "$O/calib_summary.txt" ;;
    tcc)                        # L2 hit / miss of the RHS kernels (RHS-only bench)
      timeout -k 10 300 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --output-format csv -d "$O/tcc" -o run -- python3 bench.py $A --steps 5 --warmup 1 > "$O/tcc.log" 2>&1
      python3 tools/pmc_counters.py "$O/tcc" ele_kernel riv_kernel > "$O/tcc_summary.txt" ;;
    sq) timeout -k 10 400 bash tools/sq_counters.sh "$O" > /dev/null ;;
    ode) timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/kt_ode" -o run -- python3 bench.py --no-cpu-baseline --no-et --no-many-class --no-host-vectors --e2e-ele 0 --steps 5 --warmup 1 > "$O/bench_ode_kt.json" 2> "$O/bench_ode_kt.err" ;;
    part1) timeout -k 10 300 python bench.py $A --partition-1 --steps 20 > "$O/bench_partition1.json" 2> "$O/bench_partition1.err" ;;
    rank) timeout -k 10 400 python tools/rank_timing.py > "$O/rank_timing.json" 2> "$O/rank_timing.err" ;;
    rankab:*)                   # rankab:L1,L2 -> 8-way rank timing for the production lib and each A/B lib
      libs="${step#rankab:}"
      for n in prod ${libs//,/ }; do
        if [ $n = prod ]; then L=""; else L=$PWD/shud-up_amd/build/ab/libshud_rhs_$n.so; fi
        SHUD_RHS_LIB=$L timeout -k 10 300 python tools/rank_timing.py 8 > "$O/rank8_$n.json" 2> "$O/rank8_$n.err"
      done ;;
    syn1m) timeout -k 10 900 bash tools/profile_1m.sh "$O/syn1M" > "$O/syn1M.log" 2>&1 ;;
    sizes)                      # RHS-only bench lines at other mesh sizes and in OMP semantics
      for n in 1250000 2500000 5000000; do
        timeout -k 10 300 python bench.py $A --n-ele $n --steps 100 --warmup 10 > "$O/rhs_$n.json" 2> "$O/rhs_$n.err"
      done
      timeout -k 10 300 python bench.py $A --mode omp --steps 40 --warmup 5 > "$O/rhs_omp.json" 2> "$O/rhs_omp.err" ;;
    e2e) timeout -k 10 600 bash tools/profile_e2e.sh 1000000 1 > "$O/e2e.log" 2>&1 ;;
    traj) timeout -k 10 300 python tests/diag_traj_day.py "$O/traj_ccw_day.json" > "$O/traj_ccw_day.log" 2>&1 ;;
    classes) timeout -k 10 600 python tools/class_sweep.py > "$O/class_sweep.log" 2>&1 ;;
    redbench) timeout -k 10 120 tools/ode_red_bench 31000000 30 > "$O/ode_red_bench.log" 2>&1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo done
