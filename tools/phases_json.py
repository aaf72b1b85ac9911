"""Config-2 KeyDeps phase breakdown -> profiles/<round>_config2_phases.json.

Inputs (both from one GPU box): a bench log of the product library with per-kernel timings
(ACC_BENCH_KERNELS=1 python bench.py --config 2 ...) and a log of the tuning build (tools/build_prof.sh ->
tools/ab/prof.so, -DACC_PHASE_PROF) whose stderr carries the count pass's [ct_phase] and the stream pass's [st_phase]
per-wave cycle counters. Usage: python tools/phases_json.py KERNELS_LOG PROF_LOG OUT_JSON"""
import json
import re
import sys


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise SystemExit(f"no JSON line in {path}")


def phase_lines(path, tag):
    return [ln for ln in open(path).read().splitlines() if ln.startswith(f"[{tag}]")]


def parse_avg(line):
    """'name value' pairs after 'avg cycles:' up to '|'"""
    body = line.split("avg cycles:", 1)[1].split("|", 1)[0]
    toks = body.split()
    out, i = {}, 0
    while i < len(toks) - 1:
        name, val = toks[i], toks[i + 1]
        try:
            out[name] = float(val)
            i += 2
        except ValueError:
            # multi-word names (e.g. "inline+write")
            out.setdefault(name, None)
            i += 1
    return {k: v for k, v in out.items() if v is not None}


def main():
    klog, plog, out = sys.argv[1:4]
    k = last_json(klog)
    kern = k.get("kernels_ms_per_step", {})
    ct = phase_lines(plog, "ct_phase")
    st = phase_lines(plog, "st_phase")
    waves_ct = int(re.search(r"waves=(\d+)", ct[-1]).group(1)) if ct else None
    waves_st = int(re.search(r"waves=(\d+)", st[-1]).group(1)) if st else None
    res = {
        "workload": k["config"]["workload"],
        "ms_per_step": k["ms_per_step"],
        "device_kernel_ms_per_step": k["roofline"].get("device_kernel_ms_per_step"),
        "traffic_bytes_per_step": k["roofline"].get("traffic"),
        "kernels_ms_per_step": dict(sorted(kern.items(), key=lambda kv: -kv[1])),
        "count_pass_k_v2_count": {"waves": waves_ct, "avg_cycles_per_wave": parse_avg(ct[-1]) if ct else None,
                                  "raw": ct[-1] if ct else None},
        "stream_pass_k_v3_stream": {"waves": waves_st, "avg_cycles_per_wave": parse_avg(st[-1]) if st else None,
                                    "raw": st[-1] if st else None},
        "note": "per-wave cycles from clock64() brackets in the -DACC_PHASE_PROF tuning build (same kernels, one extra "
                "store per wave); kernel ms from HIP events around each launch in the product build",
    }
    json.dump(res, open(out, "w"), indent=1)
    print(json.dumps({k2: v for k2, v in res.items() if k2 != "kernels_ms_per_step"})[:600])


if __name__ == "__main__":
    main()
