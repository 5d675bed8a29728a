#!/bin/bash
# Same-box A/B of the training step: the in-tree library vs a variant build (MST_LIB_PATH),
# alternated N times (dev tool; via gpurun).  tools/ab_lib.sh TAG VARIANT_SO [N] [extra bench args]
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
V=${2:?variant .so}
N=${3:-3}
shift 3 || true
for i in $(seq 1 "$N"); do
  for lib in "" "$V"; do
    echo "== lib ${lib:-in-tree}" >> "$OUT/ab_step.jsonl"
    MST_LIB_PATH=$lib timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 "$@" \
      >> "$OUT/ab_step.jsonl" 2>> "$OUT/ab_step.err"
  done
done
echo "ab ok"
