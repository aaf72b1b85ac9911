"""Summarise a profiles/collect.sh run into a committed per-round file.

    python profiles/summarize.py gpurun_out/prof_r04_c2 profiles/r04_config2 [--steps 9]

Writes <prefix>_kernel_stats.csv (the rocprofv3 --stats table, accord kernels first), and <prefix>_summary.json:
per-kernel average duration, per-step device time and per-step HBM traffic from the FETCH_SIZE / WRITE_SIZE
passes. FETCH_SIZE is doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B reads at 64 B) for the upper bound and kept
as is for the lower bound (`*_raw`; random gathers are not the calibrated pattern, see tools/calib_fetch.hip); KB units.
`steps` = every step the profiled bench command runs: 2 warmup + 5 timed + bench.DIAG_STEPS (2) untimed diagnostic steps
= 9 (every pipeline kernel of a step runs once per step or a fixed number of times, so totals / steps are per-step
figures). Round-3 and earlier summaries divided by 7 (the diagnostic steps were left out), overstating their per-step
figures by 9/7.
"""
import csv
import json
import os
import re
import sys
from collections import defaultdict


def short(name):
    """'void acc::rd::k_rd_stab<false>(acc::rd::View, ...)' -> 'k_rd_stab<false>'; 'acc::k_v2_count(...)' ->
    'k_v2_count'."""
    n = name[5:] if name.startswith("void ") else name
    n = n.split("(")[0]
    n = re.sub(r"\b(?:acc|rd|sh)::", "", n)
    n = re.sub(r"\s+", "", n)
    return n


def is_acc(name):
    return "acc::" in name.split("(")[0]


def load_counters(path, counter):
    tot = defaultdict(float)
    calls = defaultdict(int)
    with open(path) as f:
        for r in csv.DictReader(f):
            if r["Counter_Name"] != counter or not is_acc(r["Kernel_Name"]):
                continue
            k = short(r["Kernel_Name"])
            tot[k] += float(r["Counter_Value"]) * 1024.0
            calls[k] += 1
    return tot, calls


def main():
    src, prefix = sys.argv[1], sys.argv[2]
    steps = int(sys.argv[sys.argv.index("--steps") + 1]) if "--steps" in sys.argv else 9
    rows = list(csv.DictReader(open(os.path.join(src, "trace", "run_kernel_stats.csv"))))
    acc = [r for r in rows if is_acc(r["Name"])]
    with open(prefix + "_kernel_stats.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_ns", "avg_ns", "min_ns", "max_ns", "pct"])
        for r in acc + [r for r in rows if not is_acc(r["Name"])]:
            w.writerow([short(r["Name"]), r["Calls"],
                        r["TotalDurationNs"], r["AverageNs"], r["MinNs"], r["MaxNs"], r["Percentage"]])
    fetch, fcalls = load_counters(os.path.join(src, "fetch", "run_counter_collection.csv"), "FETCH_SIZE")
    write, wcalls = load_counters(os.path.join(src, "write", "run_counter_collection.csv"), "WRITE_SIZE")
    kernels = {}
    for r in acc:
        k = short(r["Name"])
        d = kernels.setdefault(k, dict(calls=0, total_ns=0.0))
        d["calls"] += int(r["Calls"])
        d["total_ns"] += float(r["TotalDurationNs"])
    for k, d in kernels.items():
        d["avg_ns"] = d["total_ns"] / d["calls"]
        d["ms_per_step"] = d["total_ns"] / steps / 1e6
        d["hbm_read_bytes_per_step"] = 2.0 * fetch.get(k, 0.0) / steps
        d["hbm_read_bytes_per_step_raw"] = fetch.get(k, 0.0) / steps
        d["hbm_write_bytes_per_step"] = write.get(k, 0.0) / steps
        d["hbm_read_bytes_per_launch"] = 2.0 * fetch.get(k, 0.0) / max(fcalls.get(k, 0), 1)
        d["hbm_write_bytes_per_launch"] = write.get(k, 0.0) / max(wcalls.get(k, 0), 1)
    out = dict(
        source=src, steps_profiled=steps,
        kernel_ms_per_step=sum(d["ms_per_step"] for d in kernels.values()),
        hbm_read_bytes_per_step=sum(d["hbm_read_bytes_per_step"] for d in kernels.values()),
        hbm_write_bytes_per_step=sum(d["hbm_write_bytes_per_step"] for d in kernels.values()),
        hbm_read_bytes_per_step_raw=sum(d["hbm_read_bytes_per_step_raw"] for d in kernels.values()),
        kernels=dict(sorted(kernels.items(), key=lambda kv: -kv[1]["total_ns"])),
    )
    out["hbm_bytes_per_step"] = out["hbm_read_bytes_per_step"] + out["hbm_write_bytes_per_step"]
    json.dump(out, open(prefix + "_summary.json", "w"), indent=1)
    print(json.dumps({k: v for k, v in out.items() if k != "kernels"}))


if __name__ == "__main__":
    main()
