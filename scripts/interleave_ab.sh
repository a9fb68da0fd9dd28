#!/bin/bash
# Same-box A/B of the tiled bf16 Gram's superstep order: contiguous range per wave (default) vs
# interleaved (DQ4ML_GRAM_INTERLEAVE=1), at the 8-GPU shard and at the 1e8-row headline.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
DQ4ML_GRAM_INTERLEAVE=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_determinism.py -q -m gpu \
  --timeout 120 --timeout-method thread > gpurun_out/il_tests.log 2>&1 || { tail -20 gpurun_out/il_tests.log; exit 1; }
tail -1 gpurun_out/il_tests.log
for rep in 1 2; do
  for il in 0 1; do
    echo "il=$il $(DQ4ML_GRAM_INTERLEAVE=$il N=1.25e7 timeout -k 10 300 python scripts/gram_grid_sweep.py 2>&1 | grep default)" | tee -a gpurun_out/il_ab.txt || exit 1
    echo "il=$il bench8th $(DQ4ML_GRAM_INTERLEAVE=$il timeout -k 10 300 python bench.py --steps 50 --warmup 5 --rows 1.25e7 | tail -1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))')" | tee -a gpurun_out/il_ab.txt || exit 1
    echo "il=$il bench $(DQ4ML_GRAM_INTERLEAVE=$il timeout -k 10 300 python bench.py --steps 20 --warmup 3 | tail -1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))')" | tee -a gpurun_out/il_ab.txt || exit 1
  done
done
