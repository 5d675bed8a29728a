"""Summarise rocprofv3 --pmc counter_collection.csv passes per kernel (dev tool).

usage: python tools/pmc_summary.py DIR   (reads DIR/p*/**/*counter_collection.csv)
Prints, per kernel name, the mean over dispatches of every counter collected.
"""
import collections
import csv
import glob
import sys


def main(d):
    acc = collections.defaultdict(lambda: collections.defaultdict(list))
    for f in sorted(glob.glob(f"{d}/p*/**/*counter_collection.csv", recursive=True)):
        per = collections.defaultdict(float)
        for r in csv.DictReader(open(f)):
            name = r["Kernel_Name"]
            cut = name.find(">(")
            name = name[:cut + 1] if cut >= 0 else name[:80]
            per[(name, r["Dispatch_Id"], r["Counter_Name"])] += float(r["Counter_Value"])
        for (name, _, c), v in per.items():
            acc[name][c].append(v)
    for name, cs in acc.items():
        print(name)
        for c in sorted(cs):
            v = cs[c]
            print(f"  {c:28s} {sum(v) / len(v):16.0f}  (n={len(v)})")
        g = lambda k: sum(cs[k]) / len(cs[k]) if k in cs else None  # noqa: E731
        if g("SQ_WAVE_CYCLES"):
            w = g("SQ_WAVE_CYCLES")
            for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if g(k) is not None:
                    print(f"  {k} / WAVE_CYCLES = {g(k) / w:.3f}")
        if g("SQ_VALU_MFMA_BUSY_CYCLES") and g("GRBM_GUI_ACTIVE"):
            # MFMA busy cycles summed over all SIMDs; GRBM_GUI_ACTIVE summed over 8 XCDs
            simd_cycles = g("GRBM_GUI_ACTIVE") / 8 * 1024
            print(f"  MFMA busy / SIMD-cycles = {g('SQ_VALU_MFMA_BUSY_CYCLES') / simd_cycles:.3f}")


if __name__ == "__main__":
    main(sys.argv[1])
