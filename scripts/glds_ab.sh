#!/bin/bash
# Same-box A/B of the stream Gram's DMA cache policy: nt (aux 2, the default build) vs the default
# policy (aux 0, rebuilt on the box with DQ4ML_HIPCC_EXTRA).  Every step under its own limit.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
run() { timeout -k 10 300 python bench.py --steps 10 --warmup 2 "$@" | tail -1; }
for pol in nt default nt2; do
  if [ "$pol" = default ]; then
    DQ4ML_HIPCC_EXTRA=-DDQ4ML_GLDS_AUX=0 timeout -k 10 600 python -c "from net.jgp.labs.sparkdq4ml_amd.ops import build; build.build_hip(force=True)" || exit 1
  fi
  if [ "$pol" = nt2 ]; then
    timeout -k 10 600 python -c "from net.jgp.labs.sparkdq4ml_amd.ops import build; build.build_hip(force=True)" || exit 1
  fi
  for cfg in "--dtype fp64" "--dtype fp32" "--dtype bf16 --storage fp32"; do
    echo "$pol $cfg $(run $cfg | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))')" | tee -a gpurun_out/glds_ab.txt || exit 1
  done
  echo "$pol cfg4 $(timeout -k 10 600 python benchmarks/bench_dq_pipeline.py --steps 5 --warmup 2 | tail -1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))')" | tee -a gpurun_out/glds_ab.txt || exit 1
done
