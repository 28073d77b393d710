#!/bin/bash
# One GPU session (rounds 3-4).  Steps by name, run in order; each GPU step has its own time limit and
# the chain stops at the first failure.
#   tools/gpu_session.sh TAG step [step ...]
# steps: tests faults steptests smoke driver prof deleg profc4 pmcc4 multi pmc2p pmcmulti pmcstep pmcfinal stamps
#        wsstamps4 wsstamps4noobs wsstamps4gather selfplay spprof poolsize vec policy stepmode rank2 bench poltests
#        pmcpol bench4 c4ab abl32 tanhab poltest1
set -o pipefail
TAG=${1:?tag}
shift
O=gpurun_out
mkdir -p $O
export TMPDIR=/tmp
run() {  # run NAME SECONDS CMD... ; output to $O/NAME_$TAG.{out,err}
  local name=$1 secs=$2
  shift 2
  echo "== $name"
  timeout -k 10 $secs "$@" > $O/${name}_$TAG.out 2> $O/${name}_$TAG.err
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -30 $O/${name}_$TAG.err; tail -30 $O/${name}_$TAG.out; exit 1; fi
  tail -c 1500 $O/${name}_$TAG.out
}
for step in "$@"; do
  case $step in
    tests) run pytest_gpu 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread --durations=12 ;;
    faults) run pytest_faults 400 python -u -m pytest tests/test_gpu_faults.py tests/test_gpu_env_api.py \
                tests/test_gpu_parity.py -k "fault or dealer or edited or rollout_equals" -x -v --timeout 200 --timeout-method thread ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    driver) run bench_driver 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 ;;
    prof)
      # the driver's exact command under rocprofv3: one summary row per kernel instantiation
      run prof_driver 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_driver_$TAG -o run -- \
          python3 bench.py --gpus 1 --steps 20 --warmup 5
      cp $O/prof_driver_$TAG/run_kernel_stats.csv $O/kernel_stats_driver_$TAG.csv 2>/dev/null || \
          find $O/prof_driver_$TAG -name '*kernel_stats.csv' -exec cp {} $O/kernel_stats_driver_$TAG.csv \;
      head -8 $O/kernel_stats_driver_$TAG.csv
      # the same trace averaged over the timed launches only (bench.py's region marks)
      python3 tools/trace_timed.py $(find $O/prof_driver_$TAG -name '*kernel_trace.csv' | head -1) \
          $O/prof_driver_${TAG}.err --source "rocprofv3 --kernel-trace --stats -- python3 bench.py --gpus 1 --steps 20 --warmup 5 ($TAG)" \
          --out $O/kernel_trace_timed_$TAG.json | head -60 ;;
    deleg) run deleg_ab 600 python3 tools/deleg_ab.py --rounds 12 --arms 0,6 ;;
    profc4)
      run prof_c4 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c4_$TAG -o run -- \
          python3 bench.py --no-cpu-baseline --players 4 --tables 32768
      cp $O/prof_c4_$TAG/run_kernel_stats.csv $O/kernel_stats_c4_$TAG.csv; head -5 $O/kernel_stats_c4_$TAG.csv | cut -c1-160 ;;
    pmcc4) bash tools/pmc.sh ${TAG}_4p_32768 4 32768 store all || exit 1
           bash tools/pmc.sh ${TAG}_4p_32768_inplace 4 32768 inplace traffic || exit 1 ;;
    multi)
      run bench_3p 600 python3 bench.py --no-cpu-baseline --players 3
      run bench_4p 600 python3 bench.py --no-cpu-baseline --players 4
      run bench_4p_32768 600 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 ;;
    pmc2p) bash tools/pmc.sh ${TAG}_2p 2 65536 store all || exit 1
           bash tools/pmc.sh ${TAG}_2p_inplace 2 65536 inplace traffic || exit 1
           bash tools/pmc.sh ${TAG}_2p_step 2 65536 step all || exit 1 ;;
    pmcmulti) bash tools/pmc.sh ${TAG}_3p 3 65536 store traffic || exit 1
              bash tools/pmc.sh ${TAG}_4p 4 65536 store traffic || exit 1
              bash tools/pmc.sh ${TAG}_4p_32768 4 32768 store all || exit 1 ;;
    steptests) run pytest_step 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_env_api.py \
                   tests/test_gpu_opponent_pool.py -x -v --timeout 200 --timeout-method thread ;;
    sptrace)  # kernel timeline of the config-5 dual step (pool opponent), one dual step per graph replay
      run sptrace 300 rocprofv3 --kernel-trace --output-format csv -d $O/prof_sptrace_$TAG -o run -- \
          python3 tools/bench_selfplay.py --opponent pool
      python3 tools/dual_step_timeline.py $(find $O/prof_sptrace_$TAG -name '*kernel_trace.csv' | head -1) \
          > $O/selfplay_trace_$TAG.txt && tail -14 $O/selfplay_trace_$TAG.txt ;;
    spprof) bash tools/gpu_sp_prof.sh || exit 1 ;;
    poolsize) for ps in 0 1 3 6 12; do run sps_$ps 200 python3 tools/bench_selfplay.py --opponent pool --pool-size $ps; done ;;
    pmcfinal)  # HBM traffic (FETCH_SIZE, WRITE_SIZE passes) of every kernel bench.py's lines quote, final tree
      bash tools/pmc.sh ${TAG}_2p 2 65536 store traffic || exit 1
      bash tools/pmc.sh ${TAG}_4p_32768 4 32768 store traffic || exit 1
      bash tools/pmc.sh ${TAG}_2p_step 2 65536 step traffic || exit 1 ;;
    partnertests) run pytest_partner 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_faults.py \
                      -k "partner or dealer2 or rollout_equals" -x -v --timeout 200 --timeout-method thread ;;
    partnerab)  # the C4 share (4p x 32768, six-wave dealer) with the partner hand-off off / lead 2 / lead 4, alternating
      for i in 1 2; do for ld in 0 2 4; do
        run c4_lead${ld}_$i 300 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 --only --partner-lead $ld
      done; done ;;
    partnerab3)  # lead 0 / 1 / 2, three alternations
      for i in 1 2 3; do for ld in 0 1 2; do
        run c4_lead${ld}_$i 300 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 --only --partner-lead $ld
      done; done ;;
    headab)  # the headline (2p x 65536, k_rollout_store_2p) with the partner hand-off off / lead 2 / lead 4, alternating
      for i in 1 2; do for ld in 0 2 4; do
        run head_lead${ld}_$i 300 python3 bench.py --no-cpu-baseline --only --partner-lead $ld
      done; done ;;
    leadsweep)  # the partner lead for both store kernels: headline and C4 at lead 0 / 4 / 8, alternating
      for i in 1 2; do for ld in 0 4 8; do
        run head_lead${ld}_$i 300 python3 bench.py --no-cpu-baseline --only --partner-lead $ld
        run c4_lead${ld}_$i 300 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 --only --partner-lead $ld
      done; done ;;
    stepntab)  # k_step_ws row stores non-temporal (-DSPL_STEP_OBS_NT=true, ablate/lib_stepnt.so) vs plain, alternating
      for i in 1 2 3; do
        run step_plain_$i 300 python3 bench.py --mode step --only --no-cpu-baseline --sp-tables 0
        SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_stepnt.so run step_nt_$i 300 python3 bench.py --mode step --only --no-cpu-baseline --sp-tables 0
      done ;;
    pmcstep) bash tools/pmc.sh ${TAG}_2p_step 2 65536 step all || exit 1 ;;
    stamps) run stamps 300 python3 tools/stamps.py --run ;;
    wsstamps4) WS_P=4 WS_T=32768 WS_RAW=$O/wsstamps4_raw_$TAG.npz run wsstamps4 300 python3 tools/wsstamps.py --run ;;
    wsstamps4lead)  # partner hand-off off / on (lead 2), the same stamps
      WS_LEAD=0 WS_P=4 WS_T=32768 WS_RAW=$O/wsstamps4lead0_raw_$TAG.npz run wsstamps4lead0 300 python3 tools/wsstamps.py --run
      WS_LEAD=2 WS_P=4 WS_T=32768 WS_RAW=$O/wsstamps4lead2_raw_$TAG.npz run wsstamps4lead2 300 python3 tools/wsstamps.py --run ;;
    wsstamps4noobs)  # the same without the observation stores (-DSPL_ABL=1024): is the odd-XCC lag the store path?
      WS_P=4 WS_T=32768 WS_RAW=$O/wsstamps4noobs_raw_$TAG.npz run wsstamps4noobs 300 python3 tools/wsstamps.py --run --lib splendor-gym_amd/ablate/lib_wsstamps_noobs.so ;;
    wsstamps4gather)  # the same with the deck-top / LUT gathers replaced by constants (-DSPL_ABL=16384 / 32768)
      WS_P=4 WS_T=32768 run wsstamps4nodeck 300 python3 tools/wsstamps.py --run --lib splendor-gym_amd/ablate/lib_wsstamps_nodeck.so
      WS_P=4 WS_T=32768 run wsstamps4nolut 300 python3 tools/wsstamps.py --run --lib splendor-gym_amd/ablate/lib_wsstamps_nolut.so ;;
    wsstamps2) WS_RAW=$O/wsstamps2_raw_$TAG.npz run wsstamps2 300 python3 tools/wsstamps.py --run ;;
    stepab) run bench_step 300 python3 bench.py --mode step --only --no-cpu-baseline --sp-tables 0 ;;
    abl2)  # actor timing ablation: no ring streaming (one weight chunk; wrong results by design)
      run pol_full 200 python tools/bench_policy.py --fused-only --iters 30
      SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_abl2.so run pol_abl2 200 python tools/bench_policy.py --fused-only --iters 30
      SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_abl1.so run pol_abl1 200 python tools/bench_policy.py --fused-only --iters 30
      SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_abl8.so run pol_abl8 200 python tools/bench_policy.py --fused-only --iters 30 ;;
    tanhab)  # the actor's tanh: exp form (product) vs round 3's polynomial, alternating on one box
      for i in 1 2; do
        run pol_tanhexp_$i 200 python tools/bench_policy.py --fused-only --iters 30
        SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_tanhpoly.so run pol_tanhpoly_$i 200 python tools/bench_policy.py --fused-only --iters 30
      done ;;
    foldab)  # the actor's tanh with the row factor and activation scale folded in (product) vs not (ablate/lib_prefold.so)
      for i in 1 2 3; do
        run pol_fold_$i 200 python tools/bench_policy.py --fused-only --iters 30
        SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_prefold.so run pol_prefold_$i 200 python tools/bench_policy.py --fused-only --iters 30
      done ;;
    ringab)  # the actor's ring issue (uniform wave index, buffer-resource LDS DMA) vs before (ablate/lib_prering.so)
      for i in 1 2 3; do
        run pol_ring_$i 200 python tools/bench_policy.py --fused-only --iters 30
        SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_prering.so run pol_prering_$i 200 python tools/bench_policy.py --fused-only --iters 30
      done ;;
    poltest1) run pytest_pol1 300 python -u -m pytest tests/test_gpu_policy.py -x -q --timeout 200 --timeout-method thread ;;
    selfplay) run sp_pool 300 python tools/bench_selfplay.py
              run sp_frozen 300 python tools/bench_selfplay.py --opponent frozen ;;
    bench) run bench_default 600 python3 bench.py ;;
    stepmode) run bench_step 300 python3 bench.py --mode step --only --no-cpu-baseline --sp-tables 0
              run prof_step 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_step_$TAG -o run -- \
                  python3 bench.py --mode step --only --no-cpu-baseline --sp-tables 0
              cp $O/prof_step_$TAG/run_kernel_stats.csv $O/kernel_stats_step_$TAG.csv; head -4 $O/kernel_stats_step_$TAG.csv | cut -c1-160 ;;
    rank2)  # the driver's N>1 launch rehearsed with 2 ranks on this one card (collectives over gloo)
      export SPLENDOR_DIST_BACKEND=gloo
      run bench_2rank 600 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
          --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 20 --warmup 5
      unset SPLENDOR_DIST_BACKEND ;;
    vec) run vec_step 300 python tools/bench_vec_step.py
         run prof_vec 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_vec_$TAG -o run -- python3 tools/bench_vec_step.py
         cp $O/prof_vec_$TAG/run_kernel_stats.csv $O/kernel_stats_vec_$TAG.csv; head -6 $O/kernel_stats_vec_$TAG.csv | cut -c1-200 ;;
    policy) run policy 300 python tools/bench_policy.py --iters 20 ;;
    poltests)  # the actor, pool, compact-row and dual-step GPU tests
      run pytest_pol 500 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_opponent_pool.py \
          tests/test_gpu_compact_obs.py tests/test_gpu_headline.py tests/test_gpu_parity.py tests/test_wrappers.py \
          -x -v --timeout 200 --timeout-method thread ;;
    pmcpol) bash tools/pmc_policy.sh $TAG || exit 1 ;;
    bench4) run bench_4p_32768 600 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 --only ;;
    c4ab)  # the C4 share's rollout kernels, alternating on one box: three-wave dealer vs six-wave dealer2
      for i in 1 2; do for pl in dealer dealer2; do
        run c4ab_${pl}_$i 300 python3 bench.py --no-cpu-baseline --players 4 --tables 32768 --only --pipeline $pl
      done; done ;;
    abl32) bash tools/ablate_policy32.sh || exit 1 ;;  # k_act32 timing ablations (BUILD=1 here first)
    quadtests) run pytest_quad 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_headline.py -k "quad" -x -v \
                   --timeout 300 --timeout-method thread ;;
    quadab)  # the headline shape: two-wave (4 workgroups per CU) vs quad (one per CU, partner hand-off at lead 4 / off), alternating
      for i in 1 2; do
        run head_ws_$i 300 python3 bench.py --no-cpu-baseline --only --pipeline always
        run head_quad_$i 300 python3 bench.py --no-cpu-baseline --only --pipeline quad
        run head_quad0_$i 300 python3 bench.py --no-cpu-baseline --only --pipeline quad --partner-lead 0
      done
      for f in $O/head_*_[12]_$TAG.out; do python3 -c "import json,sys; d=json.loads(open('$f').read().strip().splitlines()[-1]); r=d['roofline']; print('$f', d['value'], r['kernel'], r['kernel_us'], d.get('partner_handoffs'))"; done ;;
    chains) run step_chains 300 python3 tools/bench_step_chains.py ;;
    chainse) run step_chains_eager 300 python3 tools/bench_step_chains.py --eager --chains 1,2 --offsets 0,8000,16000,24000 ;;
    polab2)  # the fp32 actor's weight ring: LDS-DMA (product) vs VGPR-staged (lib_ringv*), hidden A prefetch 2 vs 1
      for i in 1 2; do
        run pol_full_$i 200 python tools/bench_policy.py --fused-only --iters 30
        for v in ${POLAB_LIBS:-ringv ringv_d1 d1}; do
          SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so run pol_${v}_$i 200 python tools/bench_policy.py --fused-only --iters 30
        done
      done
      for f in $O/pol_*_[12]_$TAG.out; do echo "$f $(cut -c1-120 $f)"; done ;;
    spreadab)  # the fp32 actor's ring refill: pieces in a burst behind the barrier (product) vs spread over k-steps
      SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_spread${SPREAD_K:-2}.so run pytest_spread 400 python -u -m pytest \
          tests/test_gpu_policy.py -x -q --timeout 200 --timeout-method thread
      for i in 1 2; do
        run pol_burst_$i 200 python tools/bench_policy.py --fused-only --iters 30
        for k in ${SPREAD_KS:-1 2}; do
          SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_spread$k.so run pol_spread${k}_$i 200 python tools/bench_policy.py --fused-only --iters 30
        done
      done
      for f in $O/pol_*_[12]_$TAG.out; do echo "$f $(cut -c1-160 $f)"; done ;;
    libab)  # the in-tree product library vs ablate/lib_$v.so for v in $LIBAB (policy parity on each, then alternating timings)
      for v in $LIBAB; do  # LIBAB_NOTEST=1: timing ablations (wrong results by design), no parity run
        [ "${LIBAB_NOTEST:-0}" = "1" ] || SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so run pytest_lib_$v 400 \
            python -u -m pytest tests/test_gpu_policy.py -x -q --timeout 200 --timeout-method thread
      done
      for i in 1 2; do
        run pol_product_$i 200 python tools/bench_policy.py --fused-only --iters 30
        for v in $LIBAB; do
          SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so run pol_${v}_$i 200 python tools/bench_policy.py --fused-only --iters 30
        done
      done
      for f in $O/pol_*_[12]_$TAG.out; do echo "$f $(cut -c1-160 $f)"; done ;;
    spab)  # config-5 self-play, the in-tree library's variants ablate/lib_$v.so for v in $SPAB: the pool and
           # compact-obs tests on each, then tools/bench_selfplay.py alternating (3 rounds), then a
           # dual-step timeline of the last variant
      for v in $SPAB; do  # SPAB_NOTEST=1: timing ablations (wrong results by design), no test run
        [ "${SPAB_NOTEST:-0}" = "1" ] || SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so run pytest_sp_$v 400 python -u -m pytest \
            tests/test_gpu_opponent_pool.py tests/test_gpu_compact_obs.py -x -q --timeout 200 --timeout-method thread
      done
      for i in 1 2 3; do
        for v in $SPAB; do
          SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so run sp_${v}_$i 200 python3 tools/bench_selfplay.py --opponent pool
        done
      done
      for v in ${SPAB_TRACE:-$v}; do
        SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_$v.so run spabtrace_$v 300 rocprofv3 --kernel-trace \
            --output-format csv -d $O/prof_spabtrace_${v}_$TAG -o run -- python3 tools/bench_selfplay.py --opponent pool
        python3 tools/dual_step_timeline.py $(find $O/prof_spabtrace_${v}_$TAG -name '*kernel_trace.csv' | head -1) \
            > $O/selfplay_trace_${v}_$TAG.txt && tail -14 $O/selfplay_trace_${v}_$TAG.txt
      done
      for f in $O/sp_*_[123]_$TAG.out; do echo "$f $(tail -1 $f | cut -c1-200)"; done ;;
    polab)  # the fp32 actor: staged epilogue (product) vs after each tile (ablate/lib_nopipe.so), alternating
      for i in 1 2; do
        run pol_pipe_$i 200 python tools/bench_policy.py --fused-only --iters 30
        SPLENDOR_AMD_LIB=splendor-gym_amd/ablate/lib_nopipe.so run pol_nopipe_$i 200 python tools/bench_policy.py --fused-only --iters 30
      done ;;  # step mode as 1/2/4 independent chains
    polprec) run pytest_polprec 600 python -u -m pytest tests/test_gpu_policy.py tests/test_gpu_opponent_pool.py \
                 tests/test_gpu_compact_obs.py -x -v -s --timeout 300 --timeout-method thread
             grep -h "precision_vs_float64" $O/pytest_polprec_$TAG.out > $O/precision_vs_float64_$TAG.txt || true ;;
    c5tests) run pytest_c5 600 python -u -m pytest tests/test_gpu_headline.py -k "selfplay or config5" -x -v -s \
                 --timeout 300 --timeout-method thread
             grep -h "config5_precision" $O/pytest_c5_$TAG.out > $O/config5_precision_$TAG.txt || true ;;
    faultpart) run pytest_faultpart 600 python -u -m pytest tests/test_gpu_faults.py tests/test_gpu_parity.py \
                   tests/test_gpu_headline.py -k "fault or partner or headline_rollout" -x -v --timeout 300 --timeout-method thread ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "session $TAG done"
