"""Summarise rocprofv3 --pmc passes (directories p1, p2, ... under DIR) per
kernel: the median over dispatches of every counter, plus derived ratios.

usage: python tools/pmc_summary.py DIR kernel_substring [kernel_substring ...]
"""
import csv
import glob
import os
import sys


def collect(d, kname):
    vals = {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if kname not in row.get("Kernel_Name", ""):
                continue
            c = row["Counter_Name"]
            key = (f, int(row.get("Dispatch_Id") or row.get("Correlation_Id")))
            vals.setdefault(c, {}).setdefault(key, 0.0)
            vals[c][key] += float(row["Counter_Value"])
    med = {}
    for c, per in vals.items():
        v = sorted(per.values())
        med[c] = (v[len(v) // 2], len(v))
    return med


def main():
    d = sys.argv[1]
    for k in sys.argv[2:]:
        m = collect(d, k)
        print("== %s" % k)
        for c in sorted(m):
            print("  %-28s %16.0f  (%d dispatches)" % (c, m[c][0], m[c][1]))
        g = lambda c: m.get(c, (None,))[0]
        wc = g("SQ_WAVE_CYCLES")
        if wc:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY", "SQ_ACTIVE_INST_VALU",
                      "SQ_ACTIVE_INST_LDS", "SQ_ACTIVE_INST_VMEM", "SQ_ACTIVE_INST_SCA",
                      "SQ_ACTIVE_INST_MISC", "SQ_WAIT_INST_LDS"):
                if g(c) is not None:
                    print("  %-28s %6.1f %% of wave cycles" % (c, 100.0 * g(c) / wc))
        if g("SQ_BUSY_CYCLES") and g("SQ_VALU_MFMA_BUSY_CYCLES"):
            print("  MFMA busy / SQ busy          %6.1f %%" % (100.0 * g("SQ_VALU_MFMA_BUSY_CYCLES") / g("SQ_BUSY_CYCLES")))


if __name__ == "__main__":
    main()
