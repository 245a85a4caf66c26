"""Summarise rocprofv3 --pmc passes (directories p1, p2, ... under DIR) per
kernel: the median over dispatches of every counter, plus derived ratios.

usage: python tools/pmc_summary.py [--json OUT] DIR kernel_substring [kernel_substring ...]

MFMA utilisation = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024):
GRBM_GUI_ACTIVE is summed over the 8 XCDs (MI355X_MICROARCH.md, DVFS note),
so /8 is the kernel's wall clock in shader cycles, and the MFMA busy count is
summed over all 1024 SIMDs (64 cycles per v_mfma_f64_16x16x4_f64).  With
--json the first kernel's figures go to OUT (read by bench.py).
"""
import csv
import glob
import json
import os
import sys

N_XCD = 8
N_SIMD = 256 * 4


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
    argv = sys.argv[1:]
    out = None
    if argv and argv[0] == "--json":
        out, argv = argv[1], argv[2:]
    d = argv[0]
    summary = {}
    for k in argv[1:]:
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
        util = None
        if g("GRBM_GUI_ACTIVE") and g("SQ_VALU_MFMA_BUSY_CYCLES") is not None:
            util = g("SQ_VALU_MFMA_BUSY_CYCLES") / (g("GRBM_GUI_ACTIVE") / N_XCD * N_SIMD)
            print("  MFMA utilisation             %6.1f %%  (MFMA busy / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs))"
                  % (100.0 * util))
        summary[k] = {"mfma_util": util, "counters": {c: v[0] for c, v in m.items()},
                      "dispatches": max((v[1] for v in m.values()), default=0)}
    if out and summary:
        first = next(iter(summary))
        rec = dict(summary[first], kernel=first, source_dir=d,
                   formula="SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 * 1024)")
        with open(out, "w") as f:
            json.dump(rec, f, indent=1)


if __name__ == "__main__":
    main()
