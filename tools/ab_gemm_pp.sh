#!/bin/bash
# Ping-pong GEMM A/B (dev tool, GPU box): GEMM parity tests, gemm_micro and the training-step
# bench with MST_GEMM_PP=1 (default) and 0.   tools/ab_gemm_pp.sh OUTDIR
set -e -o pipefail
OUT=${1:?outdir}; mkdir -p "$OUT"
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_bench_shapes.py -m gpu -x -q \
  --timeout 200 --timeout-method thread > "$OUT/pytest_gemm.log" 2>&1
for pp in 1 0; do
  MST_GEMM_PP=$pp timeout -k 10 120 python tools/gemm_micro.py --reps 20 > "$OUT/micro_pp$pp.txt" 2>&1
  MST_GEMM_PP=$pp timeout -k 10 120 python tools/gemm_micro.py --reps 20 --B 32 --T 15 --cin 6144 --cout 6144 > "$OUT/micro_deep_pp$pp.txt" 2>&1
done
for pp in 1 0 1 0; do
  MST_GEMM_PP=$pp timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-aux --no-cpu-baseline >> "$OUT/bench_pp$pp.jsonl" 2>> "$OUT/bench.err"
done
