"""GEMM PMC per kind (conv fwd, dgrad, wgrad) from rocprofv3 --pmc passes over bench.py (dev tool).

usage: python tools/pmc_gemm_json.py DIR OUT.json [build note]
  DIR/p*/**/*counter_collection.csv: the passes of `tools/gpu_measure.sh TAG pmcgemm`
  (SQ_VALU_MFMA_BUSY_CYCLES, SQ_INSTS_MFMA, SQ_INSTS_VALU, GRBM_GUI_ACTIVE, SQ_WAVE_CYCLES,
  SQ_WAIT_INST_ANY in one pass; rocprofv3 serialises the dispatches under --pmc).

Per kind: MFMA busy = sum of SQ_VALU_MFMA_BUSY_CYCLES / sum of SIMD-cycles (GRBM_GUI_ACTIVE is
summed over the 8 XCDs: / 8 x 1024 SIMDs), VALU:MFMA = sum SQ_INSTS_VALU / sum SQ_INSTS_MFMA,
and the issue-stall share SQ_WAIT_INST_ANY / SQ_WAVE_CYCLES. bench.py reads the newest
profiles/r*/gemm_pmc.json into its roofline object.
"""
import collections
import csv
import glob
import json
import re
import sys


def kind(name):
    if "pack_planes_kernel" in name:
        return "wgrad_pack"
    if "gemm_p_kernel" in name:
        return "wgrad"
    m = re.search(r"gemm_w_kernel<(\d+), (\d+),", name)
    if m:
        return "dgrad" if m.group(2) == "2" else "conv"
    m = re.search(r"gemm_kernel<(\d+), (true|false), (\d+),", name)
    if m:
        return "wgrad" if m.group(2) == "true" else ("dgrad" if m.group(3) == "2" else "conv")
    if "splitk_reduce" in name or "sk_fixup" in name:
        return "splitk_reduce"
    return None


def main(d, out, note=""):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        for r in csv.DictReader(open(f)):
            k = kind(r["Kernel_Name"])
            if k is None:
                continue
            tot[k][r["Counter_Name"]] += float(r["Counter_Value"])
            disp[k].add((f, r["Dispatch_Id"]))
    res = {"build": note, "source": d, "kinds": {}}
    for k, c in sorted(tot.items()):
        e = {"dispatches": len(disp[k])}
        if c.get("GRBM_GUI_ACTIVE") and "SQ_VALU_MFMA_BUSY_CYCLES" in c:
            e["mfma_busy"] = round(c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 1024), 4)
        if c.get("SQ_INSTS_MFMA"):
            e["valu_per_mfma"] = round(c.get("SQ_INSTS_VALU", 0.0) / c["SQ_INSTS_MFMA"], 3)
        if c.get("SQ_WAVE_CYCLES") and "SQ_WAIT_INST_ANY" in c:
            e["wait_inst_any"] = round(c["SQ_WAIT_INST_ANY"] / c["SQ_WAVE_CYCLES"], 4)
        e["counters"] = {n: v for n, v in sorted(c.items())}
        res["kinds"][k] = e
    with open(out, "w") as fh:
        json.dump(res, fh, indent=1)
    for k, e in res["kinds"].items():
        print(k, {x: y for x, y in e.items() if x != "counters"})


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], sys.argv[3] if len(sys.argv) > 3 else "")
