"""Print one iteration's kernel sequence (start offset, duration, gap to the
previous kernel's end) from a rocprofv3 kernel_trace.csv.
usage: python tools/trace_iter.py TRACE.csv [iteration_index_from_end] [k5_kernel_substring]"""
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
k5name = sys.argv[3] if len(sys.argv) > 3 else "k5_fused<"
k5 = [i for i, r in enumerate(rows) if k5name in r["Kernel_Name"] and "true, false" not in r["Kernel_Name"]]
back = int(sys.argv[2]) if len(sys.argv) > 2 else 5
a, b = k5[-back - 1], k5[-back]
t0 = int(rows[a]["End_Timestamp"])
prev_end = t0
tot = 0
for r in rows[a + 1:b + 1]:
    s, e = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    name = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("tritd::", "")
    print("%8.2f us  dur %8.2f  gap %6.2f  q%s  %s" % ((s - t0) / 1e3, (e - s) / 1e3, (s - prev_end) / 1e3,
                                                     r.get("Queue_Id", "?"), name[:60]))
    prev_end = max(prev_end, e)
print("K5 end -> next K5 end: %.2f us" % ((int(rows[b]["End_Timestamp"]) - t0) / 1e3))
