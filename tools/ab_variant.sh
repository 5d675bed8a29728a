#!/bin/bash
# A GEMM build variant (VAR=variants/<name>/libmst_hip.so, built with EXTRA=-D... or from another tree)
# vs the in-tree build: parity tests on the variant, then micro + bench A/B (dev tool; via gpurun).
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
V=${VAR:-variants/var/libmst_hip.so}
MST_LIB_PATH=$V timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_model.py -x -q \
  --timeout 120 --timeout-method thread -k "gemm or conv or linear or wgrad or golden or bench or splitk or stream" \
  > "$OUT/pytest_var.log" 2>&1
echo "parity ok"
timeout -k 10 300 bash tools/ab_gemm.sh "$OUT/ab_micro.txt" $V
echo "micro ok"
for lib in "" $V "" $V; do
  echo "== lib ${lib:-in-tree}" >> "$OUT/ab_bench.jsonl"
  MST_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
    >> "$OUT/ab_bench.jsonl" 2>> "$OUT/ab_bench.err"
done
echo "bench ok"
