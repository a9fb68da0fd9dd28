#!/bin/bash
# One gpurun call: kernel tests -> bench -> rocprof summary.  Stops at the first GPU fault /
# abort / timeout (rc not in {0,1}); pytest rc=1 (test failures) still lets the bench run.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {  # name timeout cmd...
  local name=$1 to=$2; shift 2
  echo "=== $name" | tee -a gpurun_out/round.log
  timeout -k 10 "$to" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a gpurun_out/round.log
  tail -15 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
STEPS=${STEPS:-"info tests bench prof"}
for s in $STEPS; do
  case $s in
    info) step info 300 python -c "import torch,sys; sys.path.insert(0,'.'); from net.jgp.labs.sparkdq4ml_amd.ops import native; print(native.hip().device_info())" ;;
    tests) step tests 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread --ignore tests/test_gpu_wide.py ;;
    alltests) step alltests 900 python -u -m pytest tests -m gpu -q --maxfail=10 --timeout 120 --timeout-method thread ;;
    rccl) step rccl 300 python -u -m pytest tests/test_gpu_rccl.py -v --timeout 120 --timeout-method thread ;;
    t) step t 600 python -u -m pytest ${TESTS} -m gpu -v --maxfail=5 --timeout 120 --timeout-method thread ;;
    widetests) step widetests 600 python -m pytest tests/test_gpu_wide.py -m gpu -q --maxfail=5 ;;
    wide16) step wide16 600 env N=2e6 D=1024 EB=16 python scripts/wide_bench.py ;;
    wide8) step wide8 900 env N=1e7 D=4096 EB=8 VARIANTS="${VARIANTS:-5:morton:8:gang}" python scripts/wide_bench.py ;;
    wide16b) step wide16b 900 env N=4e6 D=4096 EB=16 VARIANTS="${VARIANTS:-5:morton:8:gang}" python scripts/wide_bench.py ;;
    wideprof) (export TMPDIR=/tmp N=2e6 D=4096 EB=8 REPS=3; step wideprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/wideprof -o run --output-format csv -- python scripts/wide_bench.py) || exit $? ;;
    widepmc) (export TMPDIR=/tmp N=${N:-1e6} D=4096 EB=${EB:-8} REPS=${REPS:-2} VARIANTS="${VARIANTS:-5:morton:8:gang}"
       step widepmc1 600 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/widepmc1 -o run --output-format csv -- python scripts/wide_bench.py &&
       step widepmc2 600 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum -d gpurun_out/widepmc2 -o run --output-format csv -- python scripts/wide_bench.py) || exit $? ;;
    widediag) step widediag 600 env N=${N:-1e7} D=4096 EB=8 DUR=${DUR:-4} VARIANTS="${VARIANTS:-5:morton:8:gang,5:morton:82:gang,5:morton:81:gang,4:morton:8:same}" python scripts/wide_diag.py ;;
    widepmc5) (export TMPDIR=/tmp N=${N:-2e6} D=4096 EB=8 REPS=${REPS:-2} VARIANTS="${VARIANTS:-5:morton:8:gang}"
       step widepmc5a 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_INSTS_MFMA -d gpurun_out/widepmc5a -o run --output-format csv -- python scripts/wide_bench.py &&
       step widepmc5b 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM -d gpurun_out/widepmc5b -o run --output-format csv -- python scripts/wide_bench.py) || exit $? ;;
    wideshard) step wideshard 600 env DQ4ML_FORCE_COLLECTIVES=1 python benchmarks/bench_wide.py --rows 1.25e6 --steps 20 --warmup 3 --json-out gpurun_out/wideshard.json &&
               step wideshard_local 600 python benchmarks/bench_wide.py --rows 1.25e6 --steps 20 --warmup 3 --json-out gpurun_out/wideshard_local.json &&
               (export TMPDIR=/tmp DQ4ML_FORCE_COLLECTIVES=1; step wideshardprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/wideshardprof -o run --output-format csv -- python benchmarks/bench_wide.py --rows 1.25e6 --steps 10 --warmup 2) &&
               (export TMPDIR=/tmp; step wideshardprof_local 600 rocprofv3 --kernel-trace --stats -d gpurun_out/wideshardprof_local -o run --output-format csv -- python benchmarks/bench_wide.py --rows 1.25e6 --steps 10 --warmup 2) || exit $? ;;
    tailres) step tailres 600 env ROWS=${ROWS:-1.25e7} FITS=${FITS:-200} python scripts/tail_reserve_probe.py ;;
    tailresprof) (export TMPDIR=/tmp; step tailresprof 300 timeout -s KILL 240 rocprofv3 --kernel-trace -d gpurun_out/tailresprof -o run --output-format csv -- python scripts/tail_reserve_probe.py) || exit $? ;;
    cfg4) step cfg4 900 python benchmarks/bench_dq_pipeline.py --steps ${CFG4_STEPS:-5} --warmup 2 --json-out gpurun_out/cfg4.json ;;
    cfg4csv) step cfg4csv 1000 python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 5 --warmup 2 --json-out gpurun_out/cfg4csv.json &&
             (export TMPDIR=/tmp; step cfg4csvprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/cfg4csvprof -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 3 --warmup 2) &&
             step cfg4csvstream 900 env DQ4ML_FILECACHE_DEVICE_BYTES=1 python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 2 --warmup 2 --json-out gpurun_out/cfg4csvstream.json || exit $? ;;
    firstprof) step firstprof 900 env DQ4ML_BENCH_FIRST_PROFILE=gpurun_out/first.prof python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 1 --warmup 1 --json-out gpurun_out/firstprof.json &&
               step firstprof_txt 120 python -c "import pstats; s=pstats.Stats('gpurun_out/first.prof'); s.sort_stats('cumulative').print_stats(70); s.sort_stats('tottime').print_stats(40)" ;;
    cfg4csvhost) step cfg4csvhost 900 env DQ4ML_BENCH_CPROFILE=gpurun_out/cfg4csv.prof python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 3 --warmup 1 --json-out gpurun_out/cfg4csvhost.json &&
             step cfg4csvhost_txt 120 python -c "import pstats; pstats.Stats('gpurun_out/cfg4csv.prof').sort_stats('cumulative').print_stats(60)" ;;
    cfg4prof) step cfg4prof 900 env DQ4ML_BENCH_CPROFILE=gpurun_out/cfg4.prof python benchmarks/bench_dq_pipeline.py --steps 10 --warmup 2 ;;
    cfg4two) step cfg4two 900 env DQ4ML_STREAM_DQ=0 python benchmarks/bench_dq_pipeline.py --steps 5 --warmup 2 --json-out gpurun_out/cfg4two.json ;;
    kprof4sf) (export TMPDIR=/tmp; step kprof4sf 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof4sf -o run --output-format csv -- python benchmarks/bench_dq_pipeline.py --steps 3 --warmup 1) || exit $? ;;
    sf) step sf 600 python -u -m pytest tests/test_gpu_streamfuse.py -m gpu -v --maxfail=3 --timeout 120 --timeout-method thread ;;
    f32s) step f32s_t 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streamfuse.py -m gpu -q -k "fp32 or one_pass" --timeout 120 --timeout-method thread &&
          step f32s_b1 300 python bench.py --steps 20 --warmup 3 --dtype fp32 &&
          step f32s_b2 300 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
          step f32s_b3 300 python bench.py --steps 20 --warmup 3 --dtype fp32 &&
          step f32s_b4 300 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
          (export TMPDIR=/tmp; step f32spmc 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/f32spmc -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --dtype fp32split) || exit $? ;;
    f32sr) step f32sr_a 300 env DQ4ML_GRAM_STREAM_RING=2 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
           step f32sr_b 300 env DQ4ML_GRAM_STREAM_RING=3 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
           step f32sr_c 300 env DQ4ML_GRAM_STREAM_RING=2 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
           step f32sr_d 300 env DQ4ML_GRAM_STREAM_RING=3 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
           step f32sr_e 300 env DQ4ML_GRAM_STREAM_RING=2 python bench.py --steps 20 --warmup 3 --dtype fp32 || exit $? ;;
    f32s2) step f32s2_t 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_streamfuse.py tests/test_gpu_determinism.py -m gpu -q --timeout 120 --timeout-method thread &&
           step f32s2_a 300 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
           step f32s2_b 300 python bench.py --steps 20 --warmup 3 --dtype bf16 --storage fp32 &&
           step f32s2_c 300 python bench.py --steps 20 --warmup 3 --dtype fp32split &&
           step f32s2_d 300 python bench.py --steps 20 --warmup 3 --dtype bf16 --storage fp32 &&
           (export TMPDIR=/tmp; step f32s2pmc 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/f32s2pmc -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --dtype fp32split) || exit $? ;;
    qn) step qn_t 600 python -u -m pytest tests/test_gpu_owlqn.py -m gpu -v --timeout 120 --timeout-method thread &&
        step qn_b 600 python scripts/owlqn_bench.py || exit $? ;;
    pipe) step pipe_t 600 python -u -m pytest tests/test_gpu_fit_pipeline.py tests/test_gpu_pipeline.py tests/test_gpu_determinism.py tests/test_gpu_owlqn.py -m gpu -q --timeout 120 --timeout-method thread &&
          for r in 1 2; do for m in 1 2; do
            step pipe_${m}_s${r} 300 env DQ4ML_FIT_PIPELINE=$m python bench.py --steps 200 --warmup 20 --rows 1.25e7 &&
            step pipe_${m}_f${r} 300 env DQ4ML_FIT_PIPELINE=$m DQ4ML_FORCE_COLLECTIVES=1 python bench.py --steps 200 --warmup 20 --rows 1.25e7 &&
            step pipe_${m}_q${r} 300 env DQ4ML_FIT_PIPELINE=$m python bench.py --steps 100 --warmup 10 --rows 2.5e7 &&
            step pipe_${m}_h${r} 300 env DQ4ML_FIT_PIPELINE=$m python bench.py --steps 30 --warmup 5 || exit $?; done; done ;;
    pipeq) for r in 1 2; do for m in 1 2; do
            step pipeq_${m}_s${r} 300 env DQ4ML_FIT_PIPELINE=$m python bench.py --steps 200 --warmup 20 --rows 1.25e7 &&
            step pipeq_${m}_f${r} 300 env DQ4ML_FIT_PIPELINE=$m DQ4ML_FORCE_COLLECTIVES=1 python bench.py --steps 200 --warmup 20 --rows 1.25e7 || exit $?; done; done ;;
    persist) step persist_t 600 python -u -m pytest tests/test_gpu_scanfuse.py tests/test_gpu_scancut.py tests/test_gpu_semantics.py tests/test_gpu_dqvm.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread &&
          for r in 1 2; do
            step persist_w8_$r 300 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 &&
            step persist_w6_$r 300 env DQ4ML_SCAN_WPE=6 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 &&
            step persist_pc4_$r 300 env DQ4ML_SCAN_PER_CU=4 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 &&
            step persist_lb_$r 300 env DQ4ML_SCAN_GRAM_NOLB=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 || exit $?; done ;;
    cfg4ring3) step cfg4ring3 900 env DQ4ML_GRAM_STREAM_RING=3 python benchmarks/bench_dq_pipeline.py --steps 5 --warmup 2 ;;
    cfg4nodqs) step cfg4nodqs 900 env DQ4ML_DQ_STREAM=0 python benchmarks/bench_dq_pipeline.py --steps 5 --warmup 2 ;;
    gang) step gang_t 600 python -u -m pytest tests/test_gpu_wide.py -m gpu -q --maxfail=3 --timeout 120 --timeout-method thread &&
          step gang_ab 900 env N=1e7 D=4096 EB=8 REPS=5 VARIANTS="${VARIANTS:-5:morton:8:gang,4:morton:8:0:q2}" python scripts/wide_bench.py ;;
    augvalu) (export TMPDIR=/tmp
       step augvalu_t 600 python -u -m pytest tests/test_gpu_scancut.py tests/test_gpu_scanfuse.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread &&
       step augvalu_ab32 600 env VARIANTS="base;DQ4ML_CUT_AUGVALU=0;base;DQ4ML_CUT_AUGVALU=0" python scripts/cut_bench.py --features 32 --rows 2e7 &&
       step augvalu_ab64 600 env VARIANTS="base;DQ4ML_CUT_AUGVALU=0;base" python scripts/cut_bench.py --features 60 --rows 1e7) || exit $? ;;
    gangpmc) (export TMPDIR=/tmp N=2e6 D=4096 EB=8 REPS=2 VARIANTS="${VARIANTS:-5:morton:8:gang,4:morton:8:0:q2}"
       step gangpmc1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/gangpmc1 -o run --output-format csv -- python scripts/wide_bench.py &&
       step gangpmc2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum GRBM_GUI_ACTIVE -d gpurun_out/gangpmc2 -o run --output-format csv -- python scripts/wide_bench.py) || exit $? ;;
    cfg5) step cfg5 900 python benchmarks/bench_wide.py --steps ${CFG5_STEPS:-10} --warmup 2 --json-out gpurun_out/cfg5.json ;;
    csv) step csv 600 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 --json-out gpurun_out/csv.json ;;
    p10ab) for r in 1 2; do
         step p10_lds_$r 300 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 &&
         step p10_valu_$r 300 env DQ4ML_SCAN_P10=valu python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 || exit $?; done ;;
    termab) for r in 1 2 3; do
         step term_one_$r 300 python benchmarks/bench_csv_pipeline.py --steps 30 --warmup 3 &&
         step term_gen_$r 300 env DQ4ML_SCAN_TERM1=0 python benchmarks/bench_csv_pipeline.py --steps 30 --warmup 3 || exit $?; done ;;
    csvnogram) step csvnogram 600 env DQ4ML_SCAN_GRAM=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    cfg1) step cfg1 300 python benchmarks/bench_cpu_small.py --json-out gpurun_out/cfg1.json ;;
    prof4) step prof4 600 env WHICH=cfg4 python scripts/step_profile.py ;;
    prof4h) step prof4h 600 env WHICH=cfg4 ROWS=1e6 REPS=50 SORT=tottime TOP=45 python scripts/step_profile.py &&
            step prof4hc 600 env WHICH=cfg4 ROWS=1e6 REPS=50 SORT=cumulative TOP=60 python scripts/step_profile.py ;;
    proflab) step proflab 600 env WHICH=lab ROWS=1e7 REPS=100 SORT=tottime TOP=50 python scripts/step_profile.py &&
            step proflabc 600 env WHICH=lab ROWS=1e7 REPS=100 SORT=cumulative TOP=70 python scripts/step_profile.py ;;
    graphprobe) step graphprobe 300 timeout -k 10 240 python scripts/graph_probe.py ;;
    prof5) step prof5 600 env WHICH=cfg5 python scripts/step_profile.py ;;
    kprof4) (export TMPDIR=/tmp; step kprof4 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof4 -o run --output-format csv -- python benchmarks/bench_dq_pipeline.py --steps 2 --warmup 1) || exit $? ;;
    kprof5) (export TMPDIR=/tmp; step kprof5 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof5 -o run --output-format csv -- python benchmarks/bench_wide.py --steps 1 --warmup 1) || exit $? ;;
    kprofasync) (export TMPDIR=/tmp; step kprofasync 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprofasync -o run --output-format csv -- python bench.py --steps 50 --warmup 5 --rows 1.25e7 --async) || exit $? ;;
    syrkbench) step syrkbench 600 python scripts/syrk_bench.py ;;
    kprofsyrk) (export TMPDIR=/tmp CASES="1024:2000000:f64:fp64" REPS=2; step kprofsyrk 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprofsyrk -o run --output-format csv -- python scripts/syrk_bench.py) || exit $? ;;
    owlqn) step owlqn 600 python scripts/owlqn_bench.py ;;
    csvstr) step csvstr 600 python scripts/csv_strings_bench.py --rows ${CSVSTR_ROWS:-1e7} ;;
    pipedepth) for r in 1 2; do for m in 2 3 4; do
            step pipedepth_${m}_r${r} 300 env DQ4ML_FIT_PIPELINE=$m python bench.py --steps 200 --warmup 20 --rows 1.25e7 || exit $?; done; done ;;
    huber) step huber_t 300 python -u -m pytest tests/test_gpu_huber_qn.py -m gpu -q --timeout 150 --timeout-method thread &&
           step huber_dev 300 python benchmarks/bench_huber.py --steps 5 --json-out gpurun_out/huber_dev.json &&
           step huber_host 300 python benchmarks/bench_huber.py --steps 5 --host --json-out gpurun_out/huber_host.json &&
           step huber_dev_small 300 python benchmarks/bench_huber.py --steps 5 --rows 1e5 --json-out gpurun_out/huber_dev_small.json &&
           step huber_host_small 300 python benchmarks/bench_huber.py --steps 5 --rows 1e5 --host --json-out gpurun_out/huber_host_small.json &&
           (export TMPDIR=/tmp; step huber_prof 300 rocprofv3 --kernel-trace --stats -d gpurun_out/huber_prof -o run --output-format csv -- python benchmarks/bench_huber.py --steps 2) || exit $? ;;
    smoke) step smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" ;;
    bench) step bench 600 python bench.py --steps 20 --warmup 3 ;;
    benchasync) step benchasync 600 python bench.py --steps 20 --warmup 3 --async ;;
    bench8th) step bench8th 600 python bench.py --steps 50 --warmup 5 --rows 1.25e7 ;;
    bench8thasync) step bench8thasync 600 python bench.py --steps 50 --warmup 5 --rows 1.25e7 --async ;;
    bench8thrccl) step bench8thrccl 600 env DQ4ML_FORCE_COLLECTIVES=1 python bench.py --steps 50 --warmup 5 --rows 1.25e7 --async ;;
    kprof8thrccl) (export TMPDIR=/tmp DQ4ML_FORCE_COLLECTIVES=1; step kprof8thrccl 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprof8thrccl -o run --output-format csv -- python bench.py --steps 20 --warmup 5 --rows 1.25e7 --async) || exit $? ;;
    hostt) step hostt 600 python -u -m pytest tests/test_gpu_async_fit.py tests/test_gpu_fit_pipeline.py tests/test_gpu_pipeline.py tests/test_gpu_determinism.py tests/test_gpu_owlqn.py tests/test_gpu_rccl.py tests/test_gpu_scanfuse.py -m gpu -q --timeout 120 --timeout-method thread ;;
    replayab) for r in 1 2; do for m in 0 1; do
            step replay_${m}_s${r} 300 env DQ4ML_FIT_REPLAY=$m python bench.py --steps 200 --warmup 20 --rows 1.25e7 &&
            step replay_${m}_f${r} 300 env DQ4ML_FIT_REPLAY=$m DQ4ML_FORCE_COLLECTIVES=1 python bench.py --steps 200 --warmup 20 --rows 1.25e7 &&
            step replay_${m}_i${r} 300 env DQ4ML_FIT_REPLAY=$m python scripts/host_overhead.py --rows 1e5 --steps 500 || exit $?; done; done ;;
    hostprof) step hostprof 300 env HOSTOV_PROFILE=gpurun_out/hostprof python scripts/host_overhead.py --rows 1.25e7,1e5 --steps 300 ;;
    hostov) step hostov 300 python scripts/host_overhead.py && step hostovrccl 300 env DQ4ML_FORCE_COLLECTIVES=1 python scripts/host_overhead.py ;;
    f32pmc) (export TMPDIR=/tmp
       step f32pmc1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/f32pmc1 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --dtype fp32 &&
       step f32pmc2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_INST_LDS SQ_INSTS_MFMA SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d gpurun_out/f32pmc2 -o run --output-format csv -- python bench.py --steps 3 --warmup 1 --dtype fp32) || exit $? ;;
    reserveab) for r in 0 1 8 0 1 8; do step res$r 300 env DQ4ML_GRAM_RESERVE=$r python bench.py --steps 50 --warmup 5 --rows 1.25e7 --async; done
       for r in 0 1 8; do step resbig$r 300 env DQ4ML_GRAM_RESERVE=$r python bench.py --steps 20 --warmup 3; done ;;
    csvhost) step csvhost 600 env DQ4ML_BENCH_CPROFILE=gpurun_out/csv.prof python benchmarks/bench_csv_pipeline.py --rows ${CSV_ROWS:-1e7} --steps 50 --warmup 5 --json-out gpurun_out/csvhost.json &&
       python -c "import pstats; pstats.Stats('gpurun_out/csv.prof').sort_stats('tottime').print_stats(45)" > gpurun_out/csvprof_tot.txt &&
       python -c "import pstats; pstats.Stats('gpurun_out/csv.prof').sort_stats('cumulative').print_stats(60)" > gpurun_out/csvprof_cum.txt ;;
    csvhost2) step csvhost2 600 env DQ4ML_BENCH_CPROFILE=gpurun_out/csv2.prof python benchmarks/bench_csv_pipeline.py --rows ${CSV_ROWS:-1e6} --steps 500 --warmup 20 --json-out gpurun_out/csvhost2.json &&
       python -c "import pstats; pstats.Stats('gpurun_out/csv2.prof').sort_stats('tottime').print_stats(60)" > gpurun_out/csv2prof_tot.txt &&
       python -c "import pstats; pstats.Stats('gpurun_out/csv2.prof').sort_stats('cumulative').print_stats(80)" > gpurun_out/csv2prof_cum.txt ;;
    shapeprobe) step shapeprobe 180 ./scripts/mfma_shape_probe 20000 &&
       (export TMPDIR=/tmp; step shapepmc 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/shapepmc -o run --output-format csv -- ./scripts/mfma_shape_probe 5000) || exit $? ;;
    mfmapeak) step mfmapeak 120 ./scripts/mfma_peak &&
       (export TMPDIR=/tmp; step mfmapeakpmc 120 timeout -s KILL 100 rocprofv3 --kernel-trace --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_BUSY_CYCLES -d gpurun_out/mfmapeakpmc -o run --output-format csv -- ./scripts/mfma_peak) || exit $? ;;
    syrkpmc) (export TMPDIR=/tmp CASES="256:20000000:f64:fp64" REPS=2
       step syrkpmc1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE -d gpurun_out/syrkpmc1 -o run --output-format csv -- python scripts/syrk_bench.py &&
       step syrkpmc2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAIT_ANY SQ_INSTS_VMEM SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE -d gpurun_out/syrkpmc2 -o run --output-format csv -- python scripts/syrk_bench.py) || exit $? ;;
    cpubase) step cpubase 600 python scripts/cpu_baseline.py --rows 2e7 --threads 16 ;;
    scangram) for v in ${SCANABL:-0}; do step scangram$v 300 env DQ4ML_DIAG=1 DQ4ML_SCAN_ABL=$v python scripts/scan_ablation.py --gram; done && step scantable 300 python scripts/scan_ablation.py ;;
    scanabl) for v in ${SCANABL:-0 1 5 9 13 0}; do step scanabl${DQ4ML_SCAN_TICKET:-xcd}$v 300 env DQ4ML_DIAG=1 DQ4ML_SCAN_ABL=$v python scripts/scan_ablation.py; done ;;
    asynctests) step asynctests 600 python -m pytest tests/test_gpu_async_fit.py -q -m gpu ;;
    fitprof) step fitprof 300 env N=1.25e7 python scripts/fit_profile.py ;;
    dist2) step dist2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 scripts/dist_rehearsal.py ;;
    benchf32) step benchf32 600 python bench.py --steps 10 --warmup 2 --dtype fp32 ;;
    benchf32r3) step benchf32r3 600 env DQ4ML_GRAM_STREAM_RING=3 python bench.py --steps 10 --warmup 2 --dtype fp32 ;;
    benchf64) step benchf64 600 python bench.py --steps 10 --warmup 2 --dtype fp64 ;;
    benchf64old) step benchf64old 600 env DQ4ML_GRAM_STREAM=0 python bench.py --steps 10 --warmup 2 --dtype fp64 ;;
    benchf64s32) step benchf64s32 600 python bench.py --steps 10 --warmup 2 --dtype fp64 --storage fp32 ;;
    benchs32) step benchs32 600 python bench.py --steps 10 --warmup 2 --dtype bf16 --storage fp32 ;;
    benchcols) step benchcols 600 python bench.py --steps 10 --warmup 2 --dtype bf16 --storage f32cols ;;
    benchring2) step benchring2 600 env DQ4ML_GRAM_STREAM_RING=2 python bench.py --steps 10 --warmup 2 --dtype fp32 ;;
    benchring2f64) step benchring2f64 600 env DQ4ML_GRAM_STREAM_RING=2 python bench.py --steps 10 --warmup 2 --dtype fp64 ;;
    benchring2cols) step benchring2cols 600 env DQ4ML_GRAM_STREAM_RING=2 python bench.py --steps 10 --warmup 2 --dtype bf16 --storage f32cols ;;
    kprofcols) (export TMPDIR=/tmp; step kprofcols 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprofcols -o run --output-format csv -- python bench.py --steps 5 --warmup 1 --storage f32cols) || exit $? ;;
    kprofcsv) (export TMPDIR=/tmp; step kprofcsv 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprofcsv -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --steps 5 --warmup 2) || exit $? ;;
    csvtwopass) step csvtwopass 600 env DQ4ML_SCAN_LOOKBACK=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvnostream) step csvnostream 600 env DQ4ML_SCAN_STREAM=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvnt) step csvnt 600 env DQ4ML_SCAN_NT=1 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvntt) step csvntt 600 env DQ4ML_SCAN_NT=1 python -u -m pytest tests/test_gpu_scanfuse.py -q -m gpu --timeout 120 --timeout-method thread ;;
    csvlb) step csvlb 600 env DQ4ML_SCAN_GRAM_NOLB=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvnoswar) step csvnoswar 600 env DQ4ML_SCAN_SWAR=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvwpe6) step csvwpe6 600 env DQ4ML_SCAN_WPE=6 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvwpe0) step csvwpe0 600 env DQ4ML_SCAN_WPE=0 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvwpe8) step csvwpe8 600 env DQ4ML_SCAN_WPE=8 python benchmarks/bench_csv_pipeline.py --steps 20 --warmup 3 ;;
    csvpmc) (export TMPDIR=/tmp
       step csvpmc1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE -d gpurun_out/csvpmc1 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --steps 2 --warmup 1 --rows 2e7 &&
       step csvpmc2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc FETCH_SIZE -d gpurun_out/csvpmc2 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --steps 2 --warmup 1 --rows 2e7 &&
       step csvpmc3 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc WRITE_SIZE TCC_HIT_sum -d gpurun_out/csvpmc3 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --steps 2 --warmup 1 --rows 2e7) || exit $? ;;
    sweep1) step sweep1 600 env DQ4ML_FORCE_COLLECTIVES=1 python scripts/bucket_sweep.py --rows 2e6 --buckets-mb 4,16,64 ;;
    bandprof) (export TMPDIR=/tmp DQ4ML_FORCE_COLLECTIVES=1; step bandprof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/bandprof -o run --output-format csv -- python scripts/bucket_sweep.py --rows 1e6 --buckets-mb 4 --wires f32 --reps 2) || exit $? ;;
    lsq) step lsq 600 python -u -m pytest tests/test_gpu_lsq.py -m gpu -v --maxfail=5 --timeout 120 --timeout-method thread ;;
    exitprobe) (export TMPDIR=/tmp; for m in plain coop cumask; do step exitprobe_$m 200 timeout -k 10 150 rocprofv3 --kernel-trace -d gpurun_out/exitprobe_$m -o run --output-format csv -- python scripts/prof_exit_probe.py $m || exit $?; done) || exit $? ;;
    exitnoprof) for m in coop cumask; do step exitnoprof_$m 200 timeout -k 10 150 python scripts/prof_exit_probe.py $m || exit $?; done ;;
    qncrash) (export TMPDIR=/tmp DQ4ML_BENCH_AB=0; step qncrash 300 timeout -k 10 240 rocprofv3 --kernel-trace -d gpurun_out/qncrash -o run --output-format csv -- python benchmarks/bench_lbfgs.py --rows 2e5 --features 2048 --steps 1 --warmup 1) || exit $? ;;
    lbfgssmall) step lbfgssmall 600 python benchmarks/bench_lbfgs.py --rows 2e5 --features 8192 --steps 2 --warmup 1 ;;
    cfg4ov) step cfg4ov_t 600 python -u -m pytest tests/test_gpu_streamfuse.py tests/test_gpu_fit_pipeline.py -m gpu -q --timeout 120 --timeout-method thread &&
          for r in 1 2; do for m in 0 1; do
            step cfg4ov_${m}_${r} 600 env DQ4ML_STREAM_OVERLAP=$m python benchmarks/bench_dq_pipeline.py --steps 10 --warmup 2 --json-out gpurun_out/cfg4ov_${m}_${r}.json || exit $?; done; done ;;
    cutab) (export TMPDIR=/tmp
       step cutab_t 600 python -u -m pytest tests/test_gpu_scancut.py tests/test_gpu_scanfuse.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread &&
       step cutab_w32 900 env VARIANTS="${CUTV:-base}" python scripts/cut_bench.py --features 32 --rows ${CUT_ROWS:-1e8} --reps ${CUT_REPS:-5}) || exit $? ;;
    labab) (export TMPDIR=/tmp
       step labab_t 600 python -u -m pytest tests/test_gpu_scanfuse.py tests/test_gpu_scancut.py tests/test_gpu_dqvm.py tests/test_gpu_semantics.py -m gpu -q --maxfail=5 --timeout 120 --timeout-method thread &&
       step labab 900 env VARIANTS="${LABV:-base}" python scripts/cut_bench.py --rows ${LAB_ROWS:-1e8} --reps ${LAB_REPS:-20}) || exit $? ;;
    cutstamps) step cutstamps 600 env VARIANTS="base;DQ4ML_CUT_STAMPS=1" python scripts/cut_bench.py --features 32 --rows 1e8 --reps 5 ;;
    csvshard) step csvshard 600 python benchmarks/bench_csv_pipeline.py --rows 1.25e7 --steps 200 --warmup 20 --json-out gpurun_out/csvshard.json &&
              step csvshard2 600 python benchmarks/bench_csv_pipeline.py --rows 1.25e7 --steps 200 --warmup 20 --json-out gpurun_out/csvshard2.json || exit $? ;;
    x4) step lbfgs1 900 env DQ4ML_BENCH_AB=0 python benchmarks/bench_lbfgs.py --steps 3 --warmup 1 --json-out gpurun_out/lbfgs1.json &&
        step lbfgsdp 900 env DQ4ML_BENCH_AB=0 DQ4ML_FORCE_COLLECTIVES=1 python benchmarks/bench_lbfgs.py --steps 3 --warmup 1 --json-out gpurun_out/lbfgsdp.json &&
        step lbfgs1b 900 env DQ4ML_BENCH_AB=0 python benchmarks/bench_lbfgs.py --steps 3 --warmup 1 --json-out gpurun_out/lbfgs1b.json || exit $? ;;
    lbfgs) step lbfgs 900 python benchmarks/bench_lbfgs.py --steps 2 --warmup 1 --json-out gpurun_out/lbfgs.json ;;
    lbfgs8) step lbfgs8 900 python benchmarks/bench_lbfgs.py --steps 2 --warmup 1 --dtype fp8 --json-out gpurun_out/lbfgs8.json ;;
    kproflbfgs) (export TMPDIR=/tmp; step kproflbfgs 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kproflbfgs -o run --output-format csv -- python benchmarks/bench_lbfgs.py --steps 1 --warmup 0) || exit $? ;;
    cut) step cut 600 python -u -m pytest tests/test_gpu_scancut.py tests/test_gpu_scanfuse.py tests/test_gpu_dqvm.py tests/test_gpu_semantics.py -m gpu -v --maxfail=5 --timeout 120 --timeout-method thread ;;
    cutpmc) (export TMPDIR=/tmp
       step cutpmc1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/cutpmc1 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --features 32 --rows 2e7 --steps 2 --warmup 1 &&
       step cutpmc2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d gpurun_out/cutpmc2 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --features 32 --rows 2e7 --steps 2 --warmup 1) || exit $? ;;
    cutpmclab) (export TMPDIR=/tmp
       step cutpmclab1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/cutpmclab1 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --steps 2 --warmup 1 &&
       step cutpmclab2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d gpurun_out/cutpmclab2 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --steps 2 --warmup 1) || exit $? ;;
    cutabl) for ab in 0 1 2 4 7; do
         step cutabl_lab_$ab 300 env DQ4ML_DIAG=1 DQ4ML_CUT_ABLATE=$ab python benchmarks/bench_csv_pipeline.py --steps 10 --warmup 2 &&
         step cutabl_w32_$ab 300 env DQ4ML_DIAG=1 DQ4ML_CUT_ABLATE=$ab python benchmarks/bench_csv_pipeline.py --features 32 --rows 2e7 --steps 10 --warmup 2 || exit $?
       done ;;
    cutb) (export TMPDIR=/tmp
       step cutb_lab 300 env DQ4ML_DIAG=1 VARIANTS="${LABV:-base;DQ4ML_SCAN_CUT=0;DQ4ML_CUT_ABLATE=1;DQ4ML_CUT_ABLATE=4;DQ4ML_CUT_ABLATE=5}" python scripts/cut_bench.py --rows 1e8 &&
       step cutb_w32 300 env DQ4ML_DIAG=1 VARIANTS="${W32V:-base;DQ4ML_CUT_ABLATE=1;DQ4ML_CUT_ABLATE=2;DQ4ML_CUT_ABLATE=4;DQ4ML_CUT_ABLATE=7}" python scripts/cut_bench.py --features 32 --rows 2e7) || exit $? ;;
    cutpmcb) (export TMPDIR=/tmp VARIANTS=base
       step cutpmcb1 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS GRBM_GUI_ACTIVE -d gpurun_out/cutpmcb1 -o run --output-format csv -- python scripts/cut_bench.py --features 32 --rows 2e7 --reps 3 &&
       step cutpmcb2 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_ACTIVE_INST_MISC GRBM_GUI_ACTIVE -d gpurun_out/cutpmcb2 -o run --output-format csv -- python scripts/cut_bench.py --features 32 --rows 2e7 --reps 3 &&
       step cutpmcb3 300 timeout -s KILL 240 rocprofv3 --kernel-trace --pmc SQ_INST_CYCLES_VMEM SQ_ACTIVE_INST_SCA SQ_INSTS_SMEM SQ_INST_LEVEL_LDS SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/cutpmcb3 -o run --output-format csv -- python scripts/cut_bench.py --features 32 --rows 2e7 --reps 3) || exit $? ;;
    csv32s) step csv32s 600 python benchmarks/bench_csv_pipeline.py --features 32 --rows 2e7 --steps 10 --warmup 2 ;;
    cfg4csvb) step cfg4csvb 1000 python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 5 --warmup 2 --json-out gpurun_out/cfg4csvb.json ;;
    csv32) step csv32 900 python benchmarks/bench_csv_pipeline.py --features 32 --rows 1e8 --steps 10 --warmup 2 --json-out gpurun_out/csv32.json ;;
    csv64) step csv64 900 python benchmarks/bench_csv_pipeline.py --features 64 --rows ${CSV64_ROWS:-5e7} --steps 10 --warmup 2 --json-out gpurun_out/csv64.json ;;
    kprofcsv32) (export TMPDIR=/tmp; step kprofcsv32 600 rocprofv3 --kernel-trace --stats -d gpurun_out/kprofcsv32 -o run --output-format csv -- python benchmarks/bench_csv_pipeline.py --features 32 --rows 2e7 --steps 5 --warmup 2) || exit $? ;;
    prof) cd /tmp && export TMPDIR=/tmp && cd - >/dev/null; step prof 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python bench.py --steps 5 --warmup 1 ;;
  esac
done
