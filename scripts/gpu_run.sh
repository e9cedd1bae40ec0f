# GPU-box runner: bash scripts/gpu_run.sh TAG STEP [STEP ...]
# Every step runs under its own time limit; the first failing step ends the call (no retries).
# Outputs land in gpurun_out/TAG/ (merged back by gpurun).
#   test        python -m pytest tests -m gpu (whole GPU suite)
#   smoke       __graft_entry__.smoke()
#   bench_c3    python bench.py (the driver's line: C3, PMC + CPU baseline + end-to-end)
#   bench_c2 / bench_c5 / bench_dp / bench_dpn   other configs (dp = C3 Dopri5, dpn = + obs_noise 0.1)
#   prof_c3 / prof_c2 / prof_c5 / prof_dp / prof_dpn   rocprofv3 --kernel-trace --stats of kprof (30 evaluations)
set -o pipefail
TAG=$1; shift
O=gpurun_out/$TAG; mkdir -p $O
export TMPDIR=/tmp
run() {  # name seconds cmd...
  local n=$1 s=$2; shift 2
  echo "== $n ($(date +%T))"
  timeout -k 10 $s "$@" > $O/$n.log 2>&1
  local rc=$?
  echo "== $n exit $rc"
  tail -3 $O/$n.log
  return $rc
}
prof() {  # name config args...
  local n=$1 c=$2; shift 2
  # 10 warmup evaluations (GPU clocks ramp up over the first ~15 dispatches), then the 30 the summary
  # averages; the _all summary keeps every dispatch
  run $n 240 rocprofv3 --kernel-trace --stats -d $O/$n -o $n -- python3 scripts/kprof.py --warmup 10 --iters 30 \
      --config $c "$@" || return 1
  local db=$(find $O/$n -name "*.db" | head -1)
  if [ -n "$db" ]; then
    # (SKIP: dispatches of one kernel per evaluation x 10 -- the Dopri5 kernel runs twice per evaluation)
    python3 scripts/kstats_db.py $db $O/${n}_kernel_stats.csv --skip ${SKIP:-10} && python3 scripts/kstats_db.py $db $O/${n}_kernel_stats_all.csv
  else
    cp $(find $O/$n -name '*kernel_stats.csv' | head -1) $O/${n}_kernel_stats_all.csv
  fi
  head -6 $O/${n}_kernel_stats*.csv
}
pmcsq() {  # name config: one pass of SQ stall / instruction counters over kprof (2 evaluations)
  local n=$1 c=$2; shift 2
  run $n 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
      SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU -d $O/$n -o $n --output-format csv -- python3 scripts/kprof.py --iters 2 \
      --config $c "$@" || return 1
  python3 scripts/pmc_summary.py $O/$n ${KSUB:-k_} > $O/${n}.json; cat $O/${n}.json
}
pmcic() {  # name config: one pass of instruction-cache counters over kprof (2 evaluations)
  local n=$1 c=$2; shift 2
  run $n 120 timeout -s KILL 90 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE \
      -d $O/$n -o $n --output-format csv -- python3 scripts/kprof.py --iters 2 --config $c "$@" || return 1
  python3 scripts/pmc_summary.py $O/$n ${KSUB:-k_} > $O/${n}.json; cat $O/${n}.json
}
for step in "$@"; do
  case $step in
    testall) run pytest_gpu 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread || exit 1 ;;
    test) run pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    testmask) run pytest_mask 600 python -u -m pytest tests/test_gpu_acrobot_mask.py tests/test_gpu_parity.py tests/test_dopri5.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    testmaskonly) run pytest_maskonly 300 python -u -m pytest tests/test_gpu_acrobot_mask.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1 ;;
    selection) run selection 600 env MTGP_REPORT_DIR=$O python -u -m pytest tests/test_notebook_selection.py -m gpu -x -v -s --timeout 300 --timeout-method thread || exit 1 ;;
    testpin) run pytest_pin 600 python -u -m pytest tests/test_gpu_parity.py tests/test_notebook_pin.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    testcoef) run pytest_coef 600 python -u -m pytest tests/test_coefficients.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    gradtime) run gradtime 300 python scripts/grad_time.py || exit 1 ;;
    prof_grad) run prof_grad 300 rocprofv3 --kernel-trace --stats -d $O/prof_grad -o prof_grad -- python3 scripts/grad_time.py || exit 1
               python3 scripts/kstats_db.py $(find $O/prof_grad -name "*.db" | head -1) $O/prof_grad_kernel_stats.csv; head -8 $O/prof_grad_kernel_stats.csv ;;
    c5occ) run c5occ_2 300 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 || exit 1
           run c5occ_1 300 env MTGP_WIDE_LDS_MIN=90000 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 || exit 1
           run c5occ_2b 300 env MTGP_WIDE_LDS_MIN=60000 python bench.py --config c5 --no-cpu-baseline --e2e-steps 0 || exit 1 ;;
    testsched) run pytest_sched 600 python -u -m pytest tests/test_gpu_schedule.py tests/test_gpu_build.py tests/test_gpu_parity.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    testrccl) run pytest_rccl 300 python -u -m pytest tests/test_gpu_rccl.py -m gpu -x -v --timeout 240 --timeout-method thread || exit 1 ;;
    testbuild) run pytest_build 300 python -u -m pytest tests/test_gpu_build.py -m gpu -x -v --timeout 120 --timeout-method thread || exit 1 ;;
    testext) run pytest_ext 600 python -u -m pytest tests/test_gpu_ext_ops.py tests/test_gpu_build.py -m gpu -x -v --timeout 300 --timeout-method thread || exit 1 ;;
    bench_ss8) run bench_ss8 600 python bench.py --state-size 8 --steps 30 --warmup 5 --e2e-steps 0 || exit 1 ;;
    bench_ss12) run bench_ss12 600 python bench.py --state-size 12 --steps 20 --warmup 3 --e2e-steps 0 --no-cpu-baseline || exit 1 ;;
    teststate) run pytest_state 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -k state_size --timeout 300 --timeout-method thread || exit 1 ;;
    bench_c3q) run bench_c3q 300 python bench.py --no-cpu-baseline --e2e-steps 0 || exit 1 ;;
    bench_c3ext) run bench_c3ext 300 python bench.py --ext-ops --no-cpu-baseline --e2e-steps 0 || exit 1 ;;
    dbgcheck) run dbgcheck 600 env MTGP_LIB=multitreegp_amd/lib/dbg/libmtgp_hip_dbg.so python -u scripts/debug_store_check.py \
                tests/test_gpu_acrobot_mask.py tests/test_gpu_cstep.py tests/test_gpu_parity.py || exit 1 ;;
    wavetime) run wavetime 300 env MTGP_LIB=multitreegp_amd/lib/dbg/libmtgp_hip_wt.so python -u scripts/wave_times.py --save $O/wavetime.npz || exit 1
              run wavetime_nosched 300 env MTGP_LIB=multitreegp_amd/lib/dbg/libmtgp_hip_wt.so python -u scripts/wave_times.py --no-schedule || exit 1 ;;
    wavetime_fair) run wavetime_fair 300 env MTGP_FAIR=1 MTGP_LIB=multitreegp_amd/lib/dbg/libmtgp_hip_wt.so python -u scripts/wave_times.py || exit 1 ;;
    ab_fair_dp) run ab_fair_dp 600 python scripts/kvariants.py --solver dopri5 --rounds 3 --variants "prod,prod@MTGP_FAIR_DP=3" --tag dp_fair || exit 1 ;;
    ab_fair_m) run ab_fair_m 500 python scripts/kvariants.py --config c3 --rounds 6 --variants "prod@MTGP_FAIR=0,prod@MTGP_FAIR=1,prod@MTGP_FAIR=2,prod,prod@MTGP_FAIR=5" --tag c3_fair_margin || exit 1 ;;
    ab_fair_c5) run ab_fair_c5 500 python scripts/kvariants.py --config c5 --rounds 6 --variants "prod@MTGP_FAIR=0,prod" --tag c5_fair || exit 1 ;;
    ab_fair_c2) run ab_fair_c2 300 python scripts/kvariants.py --config c2 --rounds 6 --variants "prod@MTGP_FAIR=0,prod" --tag c2_fair || exit 1 ;;
    ab_fair_mode) run ab_fair_mode 500 python scripts/kvariants.py --config c3 --rounds 8 --variants "prod,prod@MTGP_FAIR_MODE=1,prod@MTGP_FAIR=9" --tag c3_fair_mode || exit 1 ;;
    ab_fair) run ab_fair 400 python scripts/kvariants.py --config c3 --rounds 8 --variants "prod,prod@MTGP_FAIR=1" --tag c3_fair || exit 1 ;;
    smoke) run smoke 180 python -c "import __graft_entry__ as g; g.smoke()" || exit 1 ;;
    bench_c3) run bench_c3 600 python bench.py || exit 1 ;;
    bench_c2) run bench_c2 600 python bench.py --config c2 || exit 1 ;;
    bench_c5) run bench_c5 600 python bench.py --config c5 || exit 1 ;;
    bench_dp) run bench_dp 600 python bench.py --solver dopri5 --steps 20 --warmup 3 || exit 1 ;;
    bench_dpn) run bench_dpn 600 python bench.py --solver dopri5 --obs-noise 0.1 --steps 10 --warmup 2 || exit 1 ;;
    prof_c3) prof prof_c3 c3 || exit 1 ;;
    prof_c3_w64) MTGP_JIT_EMIT=wave64 prof prof_c3_w64 c3 || exit 1 ;;
    prof_c3_fw) MTGP_FLAT_HALVES=0 prof prof_c3_fw c3 || exit 1 ;;
    prof_c3_h) MTGP_JIT_EMIT=halves prof prof_c3_h c3 || exit 1 ;;
    prof_c2) prof prof_c2 c2 || exit 1 ;;
    prof_c5) prof prof_c5 c5 || exit 1 ;;
    prof_dp) SKIP=20 prof prof_dp c3 --solver dopri5 || exit 1 ;;
    prof_dpn) SKIP=20 prof prof_dpn c3 --solver dopri5 --obs-noise 0.1 || exit 1 ;;
    dpab) run dpab 600 python scripts/dp_budget_ab.py || exit 1 ;;
    dpab_lpt) run dpab_lpt 600 python scripts/dp_budget_ab.py --budgets 0,16,48,128,500 --rounds 3 || exit 1 ;;
    dpab_lpt_noise) run dpab_lpt_noise 900 python scripts/dp_budget_ab.py --obs-noise 0.1 --budgets 0,16,48,128,500 --rounds 2 || exit 1 ;;
    dpab_legacy) run dpab_legacy 900 python scripts/dp_budget_ab.py --legacy-pop --budgets 0,500 --rounds 3 || exit 1 ;;
    dpab2) run dpab2 900 python scripts/dp_budget_ab.py --budgets 0,500 --rounds 3 || exit 1 ;;
    dpab_noise2) run dpab_noise2 900 python scripts/dp_budget_ab.py --obs-noise 0.1 --budgets 0,384,512,640,768 --rounds 3 || exit 1 ;;
    dpab_n500) run dpab_n500 900 python scripts/dp_budget_ab.py --obs-noise 0.1 --budgets 0,500 --rounds 3 || exit 1 ;;
    dpab_noise) run dpab_noise 900 python scripts/dp_budget_ab.py --obs-noise 0.1 --budgets 0,128,256,512 --rounds 3 || exit 1 ;;
    dptail) run dptail 600 python scripts/dp_tail.py || exit 1 ;;
    dptail_noise) run dptail_noise 600 python scripts/dp_tail.py --obs-noise 0.1 --tail 990 || exit 1 ;;
    ab_c5_union) run ab_c5_union 400 python scripts/kvariants.py --config c5 --rounds 6 --variants "prod,prod@MTGP_JIT_LDS_PIPE=1" --tag c5_union || exit 1 ;;
    dpprof) run dpprof 700 bash scripts/dpprof.sh || exit 1 ;;
    ab_c5_mse) run ab_c5_mse 400 python scripts/kvariants.py --config c5 --rounds 6 --variants "prod,mseall,noprog" --tag c5_mse || exit 1 ;;
    ab_c3_noprog) run ab_c3_noprog 400 python scripts/kvariants.py --config c3 --rounds 6 --variants "prod,noprog" --tag c3_noprog || exit 1 ;;
    ab_dp_waves) run ab_dp_waves 600 python scripts/kvariants.py --solver dopri5 --rounds 4 --variants "prod,dpw3,dpw4" --tag dp_waves || exit 1 ;;
    ab_dpn_waves) run ab_dpn_waves 600 python scripts/kvariants.py --solver dopri5 --obs-noise 0.1 --rounds 3 --variants "prod,dpw3,dpw4" --tag dpn_waves || exit 1 ;;
    ab_c5_merge) run ab_c5_merge 400 python scripts/kvariants.py --config c5 --rounds 6 --variants "prod,premerge" --tag c5_merge || exit 1 ;;
    ab_c3_merge) run ab_c3_merge 400 python scripts/kvariants.py --config c3 --rounds 6 --variants "prod,premerge" --tag c3_merge || exit 1 ;;
    ab_c5_bfm) run ab_c5_bfm 400 python scripts/kvariants.py --config c5 --rounds 6 --variants "prod,shift" --tag c5_bfm || exit 1 ;;
    ab_c3_bfm) run ab_c3_bfm 400 python scripts/kvariants.py --config c3 --rounds 8 --variants "prod,shift" --tag c3_bfm || exit 1 ;;
    ab_c2_noprog) run ab_c2_noprog 400 python scripts/kvariants.py --config c2 --rounds 6 --variants "prod,noprog" --tag c2_noprog || exit 1 ;;
    ab_c2_merge) run ab_c2_merge 400 python scripts/kvariants.py --config c2 --rounds 10 --variants "prod,nomerge" --tag c2_merge || exit 1 ;;
    ab_c2_fuse) run ab_c2_fuse 400 python scripts/kvariants.py --config c2 --rounds 10 --variants "prod,nofuse" --tag c2_fuse || exit 1 ;;
    ab_c2) V=prod; for f in multitreegp_amd/lib/abrun/libmtgp_hip_*.so; do b=$(basename $f .so); V=$V,${b#libmtgp_hip_}; done
      run ab_c2 400 python scripts/kvariants.py --config c2 --rounds 8 --variants $V --tag ab_c2 || exit 1 ;;
    bench_gloo2) run bench_gloo2 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --dist-backend gloo --steps 10 --warmup 2 --no-pmc --e2e-steps 3 || exit 1 ;;
    rccl2) run rccl2 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 scripts/rccl_two_ranks.py || exit 1 ;;
    ab_dp_layout) run ab_dp_layout 600 python scripts/kvariants.py --solver dopri5 --rounds 4 --variants "prod@MTGP_TRAJ_LAYOUT=time,prod" --tag dp_layout || exit 1 ;;
    ab_dpw3) run ab_dpw3 600 python scripts/kvariants.py --solver dopri5 --rounds 4 --variants "prod,dpw3" --tag dp_w3 && run ab_dpw3n 600 python scripts/kvariants.py --solver dopri5 --obs-noise 0.1 --rounds 2 --variants "prod,dpw3" --tag dpn_w3 || exit 1 ;;
    listctr) run listctr 120 rocprofv3 -L || exit 1 ;;
    fbcount) run fbcount 300 python scripts/fb_count.py || exit 1 ;;
    ab_c3) V=prod; for f in multitreegp_amd/lib/abrun/libmtgp_hip_*.so; do b=$(basename $f .so); V=$V,${b#libmtgp_hip_}; done
      V=${V/,fbcount/}
      run ab_c3 600 python scripts/kvariants.py --config c3 --rounds 6 --variants $V --tag ab_c3 || exit 1 ;;
    budget)  # C3 per-section budget: interleaved timing of every lib/abrun variant, then one SQ pass each
      V=prod; for f in multitreegp_amd/lib/abrun/libmtgp_hip_*.so; do b=$(basename $f .so); V=$V,${b#libmtgp_hip_}; done
      run budget_time 600 python scripts/kvariants.py --config c3 --rounds 4 --variants $V --tag budget || exit 1
      for v in ${V//,/ }; do
        L=multitreegp_amd/lib/libmtgp_hip.so; [ $v != prod ] && L=multitreegp_amd/lib/abrun/libmtgp_hip_$v.so
        run budget_pmc_$v 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY \
          SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM -d $O/budget_pmc_$v -o pmc --output-format csv -- \
          python3 scripts/kprof.py --iters 2 --config c3 --lib $L || exit 1
        python3 scripts/pmc_summary.py $O/budget_pmc_$v k_ctl_dynamic > $O/budget_pmc_$v.json; cat $O/budget_pmc_$v.json
      done ;;
    pmc_fair)  # FETCH / WRITE of k_ctl_dynamic with the FairShare table off (MTGP_FAIR=0) and on (default)
      for f in 0 3; do
        for c in FETCH_SIZE WRITE_SIZE; do
          run pmc_fair${f}_$c 120 env MTGP_FAIR=$f timeout -s KILL 90 rocprofv3 --pmc $c -d $O/pmc_fair${f}_$c -o pmc \
            --output-format csv -- python3 scripts/kprof.py --iters 2 --config c3 || exit 1
          python3 scripts/pmc_summary.py $O/pmc_fair${f}_$c k_ctl_dynamic > $O/pmc_fair${f}_$c.json; cat $O/pmc_fair${f}_$c.json
        done
      done ;;
    pmcsq_flat) KSUB=k_flatten_wave pmcsq pmcsq_flat c3 && python3 scripts/pmc_summary.py $O/pmcsq_flat k_jit_emit_waves > $O/pmcsq_emit.json && cat $O/pmcsq_emit.json || exit 1 ;;
    pmcmem_flat) run pmcmem_flat 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_INSTS_SMEM SQ_INSTS_VMEM_RD \
        SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_BRANCH -d $O/pmcmem_flat -o pmcmem_flat --output-format csv \
        -- python3 scripts/kprof.py --iters 2 --config c3 || exit 1
      python3 scripts/pmc_summary.py $O/pmcmem_flat k_flatten_wave > $O/pmcmem_flat.json && cat $O/pmcmem_flat.json
      python3 scripts/pmc_summary.py $O/pmcmem_flat k_jit_emit_waves > $O/pmcmem_emit.json && cat $O/pmcmem_emit.json || exit 1 ;;
    pmcsq_flat5) KSUB=k_flatten_wave pmcsq pmcsq_flat5 c5 && python3 scripts/pmc_summary.py $O/pmcsq_flat5 k_jit_emit_groups > $O/pmcsq_emit5.json && cat $O/pmcsq_emit5.json || exit 1 ;;
    pmcmem_c3) run pmcmem_c3 120 timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_VMEM_RD \
        SQ_INSTS_VMEM_WR SQ_INSTS_FLAT SQ_INSTS_SMEM SQ_INSTS_LDS -d $O/pmcmem_c3 -o pmcmem_c3 --output-format csv \
        -- python3 scripts/kprof.py --iters 2 --config c3 || exit 1
      python3 scripts/pmc_summary.py $O/pmcmem_c3 k_ctl_dynamic > $O/pmcmem_c3.json && cat $O/pmcmem_c3.json || exit 1 ;;
    pmcsq_c5) KSUB=k_sr_wide pmcsq pmcsq_c5 c5 || exit 1 ;;
    pmcsq_c3) KSUB=k_ctl_dynamic pmcsq pmcsq_c3 c3 || exit 1 ;;
    pmcsq_c2) KSUB=k_ctl_static pmcsq pmcsq_c2 c2 || exit 1 ;;
    pmcic_c5) KSUB=k_sr_wide pmcic pmcic_c5 c5 || exit 1 ;;
    pmcic_c3) KSUB=k_ctl_dynamic pmcic pmcic_c3 c3 || exit 1 ;;
    pmcic_c2) KSUB=k_ctl_static pmcic pmcic_c2 c2 || exit 1 ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "all steps done"
