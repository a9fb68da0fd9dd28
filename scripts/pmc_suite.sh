#!/bin/bash
# Counter evidence for the hot kernels (VERDICT r4 "next" #7): every workload runs twice under
# rocprofv3 --pmc, one pass per counter group (a pass may hold at most 4 TCC / 8 SQ / 2 GRBM slots,
# and FETCH_SIZE takes 3 TCC ones), each pass under its own hard time limit.  Summaries:
#   python scripts/pmc_report.py gpurun_out/pmc_<name>_{a,b} --kernel <substring>
# Workloads (PMC_SET): lsq (lsq_qn_kernel, the one-launch 1e6 x 16384 bf16 l-bfgs fit), cut (dq_scan_cut, the 77 GB config-4 CSV),
# cut32 (dq_scan_cut, the BASELINE-shape 1e8 x 32 CSV), span (csv_span_eq, string column filter), tall (centred gram_tall_bf16_kernel, the headline),
# wide (gram_wide_gang_kernel, config 5 at 2e6 rows).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
# (bench_lbfgs: no host-steered A/B fit; the one-launch lsq_qn_kernel is profiled whole -- its
# launch is a plain co-resident grid since round 6, the cooperative launch that crashed the
# profiler's teardown at exit is gone: profiles/r6_coop_exit.md)
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0 DQ4ML_BENCH_AB=0
A="GRBM_GUI_ACTIVE FETCH_SIZE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_VMEM SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY"
B="GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum SQ_INSTS_LDS SQ_ACTIVE_INST_VALU"
run() {  # name seconds kernel-regex cmd...  (counters only for the matching kernels: the 64 MiB
  local name=$1 to=$2 kre=$3; shift 3  # limit on what a call copies back)
  for pass in a b; do
    local ctr=$A
    [ $pass = b ] && ctr=$B
    echo "=== pmc $name $pass"
    timeout -s KILL "$to" rocprofv3 --kernel-trace --pmc $ctr --kernel-include-regex "$kre" \
      -d "gpurun_out/pmc_${name}_$pass" -o run --output-format csv -- "$@" > "gpurun_out/pmc_${name}_$pass.log" 2>&1
    local rc=$?
    tail -2 "gpurun_out/pmc_${name}_$pass.log"
    if [ $rc -ne 0 ]; then echo "pmc $name $pass rc=$rc"; exit $rc; fi
  done
}
for w in ${PMC_SET:-wide tall span cut lsq}; do
  case $w in
    lsq) run lsq 240 lsq_qn_kernel python benchmarks/bench_lbfgs.py --steps 1 --warmup 1 ;;
    cut) run cut 420 dq_scan_cut python benchmarks/bench_csv_pipeline.py --features 64 --rows 1.25e8 --steps 2 --warmup 1 ;;
    cut32) run cut32 420 dq_scan_cut python benchmarks/bench_csv_pipeline.py --features 32 --rows 1e8 --steps 2 --warmup 1 ;;
    span) run span 240 csv_span_eq python scripts/span_bench.py --rows 1e7 ;;
    tall) run tall 240 gram_tall_bf16 python bench.py --steps 10 --warmup 3 ;;
    wide) (export N=2e6 D=4096 EB=8 REPS=2; run wide 240 gram_wide_gang python scripts/wide_bench.py) || exit $? ;;  # (no env hop after --)
  esac
done
