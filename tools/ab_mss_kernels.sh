#!/bin/bash
# Same-box per-kernel A/B of the multi-scale loss (dev tool; via gpurun from the repo root):
# rocprofv3 --kernel-trace --stats over bench_aux.py --workload mss, alternating the in-tree
# library with VAR (default variants/prev/libmst_hip.so), ROUNDS rounds (2); prints the mss_*
# kernels' average durations per run.
#   tools/ab_mss_kernels.sh TAG
set -e -o pipefail
OUT=gpurun_out/${1:?tag}; mkdir -p "$OUT"
V=${VAR:-variants/prev/libmst_hip.so}
export TMPDIR=/tmp
n=0
for r in $(seq 1 ${ROUNDS:-2}); do
  for lib in "" $V; do
    n=$((n + 1))
    MST_LIB_PATH=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$OUT/p$n" -o run -- python3 bench_aux.py --workload mss --no-cpu-baseline \
      > "$OUT/run$n.log" 2>&1
    f=$(find "$OUT/p$n" -name "*kernel_stats.csv" | head -1)
    echo "== run $n lib ${lib:-in-tree}" >> "$OUT/summary.txt"
    python3 - "$f" >> "$OUT/summary.txt" <<'PY'
import csv, sys
for r in csv.DictReader(open(sys.argv[1])):
    if 'mss_' in r['Name']:
        print(f"  {float(r['AverageNs']) / 1e3:9.1f} us  x{r['Calls']:>4}  {r['Name'][:70]}")
PY
  done
done
cat "$OUT/summary.txt"
