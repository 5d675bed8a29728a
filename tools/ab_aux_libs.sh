#!/bin/bash
# Same-box A/B of one bench_aux workload across library builds (dev tool; via gpurun).
#   tools/ab_aux_libs.sh TAG WORKLOAD N LIB1 [LIB2 ...]   ("" or "-" = in-tree)
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
W=${2:?workload}; N=${3:?reps}; shift 3
for i in $(seq 1 "$N"); do
  for lib in "$@"; do
    [ "$lib" = "-" ] && lib=""
    echo "== lib ${lib:-in-tree}" >> "$OUT/ab_aux.jsonl"
    MST_LIB_PATH=$lib timeout -k 10 200 python -u bench_aux.py --workload "$W" --no-cpu-baseline --no-parity \
      >> "$OUT/ab_aux.jsonl" 2>> "$OUT/ab_aux.err"
  done
done
echo "ab ok"
