"""Print the kernel timeline of the last full step of a rocprofv3 --kernel-trace CSV (gaps, overlaps, queues).

    python tools/timeline.py gpurun_out/<dir>/trace/run_kernel_trace.csv [first-kernel-substring]
"""
import csv
import sys

path = sys.argv[1]
marker = sys.argv[2] if len(sys.argv) > 2 else "prep_txn"
rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
idx = [i for i, r in enumerate(rows) if marker in r["Kernel_Name"]]
s, e = (idx[-2], idx[-1]) if len(idx) >= 2 else (0, len(rows))
t0 = int(rows[s]["Start_Timestamp"])
prev_end = t0
busy = 0
for r in rows[s:e]:
    st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
    print(f"{(st - t0) / 1000:8.1f} {(en - st) / 1000:7.1f} gap {(st - prev_end) / 1000:6.1f} q{r['Queue_Id']} "
          f"g{r['Grid_Size_X']}x{r['Workgroup_Size_X']} {r['Kernel_Name'][:70]}")
    prev_end = max(prev_end, en)
print(f"step span {(prev_end - t0) / 1000:.1f} us, {e - s} dispatches")
