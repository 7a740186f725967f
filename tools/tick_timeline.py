"""Per-tick kernel timeline of the RCCL tick transport from a rocprofv3
kernel trace (tools/gpu_tickprof2.sh): durations of the seal kernel and the
allgather's kernel, and the gaps between them, over ticks that ran back to back.

    python tools/tick_timeline.py <kernel_trace.csv> [--out profiles/x.json]
"""
import argparse
import csv
import json
import statistics


def pct(v, q):
    v = sorted(v)
    return v[min(len(v) - 1, int(q * (len(v) - 1) + 0.5))] if v else None


def summary(v):
    if not v:
        return None
    return {"n": len(v), "p50_us": round(pct(v, 0.5), 2), "p10_us": round(pct(v, 0.1), 2),
            "p90_us": round(pct(v, 0.9), 2), "mean_us": round(statistics.fmean(v), 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--out", default="")
    ap.add_argument("--burst-gap-us", type=float, default=30.0,
                    help="a gap longer than this ends a burst of back-to-back ticks")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    ks = []
    for r in rows:
        name = r.get("Kernel_Name", "")
        ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), name, r.get("Queue_Id", ""),
                   r.get("Process_Id", r.get("Pid", ""))))
    ks.sort()
    names = {}
    for k in ks:
        names[k[2]] = names.get(k[2], 0) + 1
    seal = [k for k in ks if "tick_seal" in k[2]]
    seal_d = [(k[1] - k[0]) / 1e3 for k in seal]
    # the kernel that follows each seal on its queue is the allgather's
    by_q = {}
    for k in ks:
        by_q.setdefault((k[4], k[3]), []).append(k)
    coll_d, gap_sc, gap_cs, period = [], [], [], []
    coll_names = {}
    for q, lst in by_q.items():
        for i, k in enumerate(lst):
            if "tick_seal" not in k[2] or i + 1 >= len(lst):
                continue
            c = lst[i + 1]
            coll_names[c[2]] = coll_names.get(c[2], 0) + 1
            coll_d.append((c[1] - c[0]) / 1e3)
            g = (c[0] - k[1]) / 1e3
            if g < a.burst_gap_us:
                gap_sc.append(g)
            if i + 2 < len(lst) and "tick_seal" in lst[i + 2][2]:
                g2 = (lst[i + 2][0] - c[1]) / 1e3
                if g2 < a.burst_gap_us:
                    gap_cs.append(g2)
                    period.append((lst[i + 2][0] - k[0]) / 1e3)
    out = {
        "kernels": names,
        "collective_kernel": coll_names,
        "seal_us": summary(seal_d),
        "collective_us": summary(coll_d),
        "gap_seal_end_to_collective_start_us": summary(gap_sc),
        "gap_collective_end_to_next_seal_start_us": summary(gap_cs),
        "tick_period_back_to_back_us": summary(period),
    }
    print(json.dumps(out, indent=1))
    if a.out:
        with open(a.out, "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
