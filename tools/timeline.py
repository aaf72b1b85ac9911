"""Print one call's kernel / copy timeline from a rocprofv3 --kernel-trace [--memory-copy-trace] csv pair: every
kernel with its start offset, duration and the idle gap before it on its queue (host syncs show as gaps).
usage: timeline.py <dir>/<prefix> <first-kernel-substring> <occurrence> [<stop-substring>]"""
import csv
import os
import re
import sys

base, first, occ = sys.argv[1], sys.argv[2], int(sys.argv[3])
stop = sys.argv[4] if len(sys.argv) > 4 else first
rows = [dict(r, kind="K") for r in csv.DictReader(open(base + "_kernel_trace.csv"))]
if os.path.exists(base + "_memory_copy_trace.csv"):
    for r in csv.DictReader(open(base + "_memory_copy_trace.csv")):
        rows.append(dict(r, kind="C", Kernel_Name="copy " + r.get("Direction", ""), Queue_Id="copy"))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if r["kind"] == "K" and first in r["Kernel_Name"]]
i0 = starts[occ]
i1 = next((i for i in range(i0 + 1, len(rows)) if rows[i]["kind"] == "K" and stop in rows[i]["Kernel_Name"]), len(rows))
t0 = int(rows[i0]["Start_Timestamp"])
last_end = t0
busy = 0
for r in rows[i0:i1]:
    s, e = int(r["Start_Timestamp"]) - t0, int(r["End_Timestamp"]) - t0
    nm = re.sub(r"\(.*", "", r["Kernel_Name"]).replace("void ", "").replace("acc::", "")[:40]
    gap = s - last_end
    last_end = max(last_end, e)
    busy += e - s
    print(f"{r['Queue_Id']:>5} {s / 1000:9.1f} {(e - s) / 1000:8.1f}us gap {gap / 1000:7.1f} {nm}")
print("span us %.1f busy us %.1f" % ((last_end) / 1000, busy / 1000))
