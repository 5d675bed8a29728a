#!/bin/bash
# Two rocprofv3 --pmc passes (SQ issue/wait counters; LDS/TCC counters) over any python command,
# then a per-kernel summary. Dev tool.
#   tools/pmc_cmd.sh OUTDIR script.py [args...]
set -e -o pipefail
OUT=${1:?outdir}; shift
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE"
P2="SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS TCC_HIT TCC_MISS"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 180 rocprofv3 --pmc $P --output-format csv -d "$OUT/p$i" -o run -- \
    python3 "$@" > "$OUT/p$i.log" 2>&1
done
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.txt"
