#!/bin/bash
# A/B a GEMM variant library against the in-tree one on tools/gemm_micro.py shapes (dev tool).
#   tools/ab_gemm.sh OUTFILE VARIANT_SO [VARIANT_SO...]
set -e -o pipefail
OUT=${1:?out}; shift
mkdir -p "$(dirname "$OUT")"
SHAPES=("--T 126 --cin 2048 --cout 2048" "--T 252 --cin 1536 --cout 1536" "--T 15 --cin 4096 --cout 6144" "--T 63 --cin 2048 --cout 3072")
for lib in "" "$@"; do
  echo "== lib ${lib:-in-tree}" >> "$OUT"
  for s in "${SHAPES[@]}"; do
    MST_LIB_PATH=$lib timeout -k 10 120 python tools/gemm_micro.py --reps 10 $s >> "$OUT" 2>&1
  done
done
