#!/bin/bash
# Same-box A/B of the config-5 SYRK between this tree and a second built tree ($AB_OLD, default
# abtree/): alternating wide_diag runs (time + board power), then one PMC pass pair per tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OLD=${AB_OLD:-abtree}
V=${AB_VARIANTS:-5:morton:8:gang}
mkdir -p gpurun_out
for rep in 1 2; do
  for tree in "$OLD" .; do
    echo "=== $tree rep $rep"
    (cd "$tree" && timeout -k 10 240 env N=1e7 D=4096 EB=8 DUR=4 VARIANTS="$V" python scripts/wide_diag.py) || exit $?
  done
done 2>&1 | grep -v amdgpu.ids | tee gpurun_out/ab_wide.log
[ "${PIPESTATUS[0]}" -eq 0 ] || exit 1
export TMPDIR=/tmp
for tree in "$OLD" .; do
  tag=$(basename "$(cd "$tree" && pwd)")
  (cd "$tree" && timeout -s KILL 200 env N=2e6 D=4096 EB=8 REPS=2 VARIANTS="$V" rocprofv3 --kernel-trace --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCP_TCC_READ_REQ_sum SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES -d "$GRAFT_REPO_ROOT/gpurun_out/abpmc_$tag" -o run --output-format csv -- python scripts/wide_bench.py > "$GRAFT_REPO_ROOT/gpurun_out/abpmc_$tag.log" 2>&1) || exit $?
done
