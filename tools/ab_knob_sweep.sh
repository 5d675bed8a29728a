#!/bin/bash
# Same-box sweep of one knob over several values, alternated N times (dev tool; via gpurun).
#   tools/ab_knob_sweep.sh TAG VAR "v1 v2 ..." [N]
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
VAR=${2:?var}; VALS=${3:?values}; N=${4:-2}
for i in $(seq 1 "$N"); do
  for v in $VALS; do
    echo "== $VAR=$v" >> "$OUT/sweep.jsonl"
    env "$VAR=$v" timeout -k 10 200 python -u bench.py --no-aux --no-cpu-baseline --steps 20 --warmup 3 \
      >> "$OUT/sweep.jsonl" 2>> "$OUT/sweep.err"
  done
done
echo "sweep ok"
