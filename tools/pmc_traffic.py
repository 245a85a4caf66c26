"""Turn rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into HBM bytes per
launch of the fused update kernel (k5_fused<RP,false>).

Corrections (MI355X_MICROARCH.md §HBM): on gfx950 FETCH_SIZE reports half of
the bytes of a wide (16 B/lane) coalesced streaming read -> x2; WRITE_SIZE is
exact for 16-B streaming stores.  Both counters are in KiB.

usage: python tools/pmc_traffic.py FETCH_DIR WRITE_DIR OUT.json [algorithmic_bytes [kernel [first:last]]]
(first:last: only dispatches first..last-1 in dispatch order, e.g. the bench's
timed window; default all.  The config-5 solve densifies E after ~30
iterations, so its later dispatches move more bytes than the timed window's.)
(kernel: a substring of the kernel name, default "k5_fused<64, false", which matches
the stored-Y_O and the derived-Y_O instantiations)
"""
import csv
import glob
import json
import os
import sys


def per_dispatch(d, counter, kname="k5_fused<64, false"):
    files = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    vals = {}
    for f in files:
        for row in csv.DictReader(open(f)):
            if kname not in row.get("Kernel_Name", ""):
                continue
            if row.get("Counter_Name") != counter:
                continue
            key = int(row.get("Dispatch_Id") or row.get("Correlation_Id"))
            vals[key] = vals.get(key, 0.0) + float(row["Counter_Value"])
    return [vals[k] for k in sorted(vals)]  # dispatch order


def main():
    fd, wd, out = sys.argv[1:4]
    alg = float(sys.argv[4]) if len(sys.argv) > 4 else None
    kname = sys.argv[5] if len(sys.argv) > 5 else "k5_fused<64, false"
    fetch = per_dispatch(fd, "FETCH_SIZE", kname)
    write = per_dispatch(wd, "WRITE_SIZE", kname)
    window = None
    if len(sys.argv) > 6:
        a, b = (int(x) for x in sys.argv[6].split(":"))
        fetch, write, window = fetch[a:b], write[a:b], [a, b]
    if not fetch or not write:
        raise SystemExit("no k5 dispatches found")
    med = lambda v: sorted(v)[len(v) // 2]
    f_kib, w_kib = med(fetch), med(write)
    total = (2.0 * f_kib + w_kib) * 1024.0
    res = {"kernel": kname, "dispatches": [len(fetch), len(write)], "window": window,
           "FETCH_SIZE_KiB_median": f_kib, "WRITE_SIZE_KiB_median": w_kib,
           "read_bytes_corrected": 2.0 * f_kib * 1024.0, "write_bytes": w_kib * 1024.0,
           "bytes_per_launch": total,
           "correction": "FETCH_SIZE x2 (gfx950 wide-stream undercount), WRITE_SIZE x1"}
    if alg:
        res["algorithmic_bytes"] = alg
        res["traffic_over_algorithmic"] = total / alg
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
