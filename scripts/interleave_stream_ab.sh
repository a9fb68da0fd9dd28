#!/bin/bash
# Same-box A/B of the stream Gram kernels' stage order (interleaved default vs contiguous ranges).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" && mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_determinism.py tests/test_gpu_pipeline.py \
  tests/test_gpu_dqvm.py -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/ils_tests.log 2>&1 || { tail -20 gpurun_out/ils_tests.log; exit 1; }
tail -1 gpurun_out/ils_tests.log
ms() { tail -1 | python -c 'import json,sys; print(round(json.loads(sys.stdin.read())["ms_per_step"],4))'; }
for rep in 1 2; do
  for il in 0 1; do
    echo "il=$il f64 $(DQ4ML_GRAM_INTERLEAVE=$il timeout -k 10 300 python bench.py --steps 10 --warmup 2 --dtype fp64 | ms)" \
         "f32 $(DQ4ML_GRAM_INTERLEAVE=$il timeout -k 10 300 python bench.py --steps 10 --warmup 2 --dtype fp32 | ms)" \
         "s32 $(DQ4ML_GRAM_INTERLEAVE=$il timeout -k 10 300 python bench.py --steps 10 --warmup 2 --dtype bf16 --storage fp32 | ms)" \
         "cfg4 $(DQ4ML_GRAM_INTERLEAVE=$il timeout -k 10 600 python benchmarks/bench_dq_pipeline.py --steps 5 --warmup 2 | ms)" \
         | tee -a gpurun_out/ils_ab.txt || exit 1
  done
done
