#!/bin/bash
# Same-box A/B: Adam per bucket inside backward (the default) vs one launch in opt.step()
# (--adam-step), alternated N times (dev tool; via gpurun).  tools/ab_adam_overlap.sh TAG [N]
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
N=${2:-3}
for i in $(seq 1 "$N"); do
  for k in "" "--adam-step"; do
    echo "== ${k:-default}" >> "$OUT/ab.jsonl"
    timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 $k >> "$OUT/ab.jsonl" 2>> "$OUT/ab.err"
  done
done
echo "ab ok"
