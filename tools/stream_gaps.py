"""Where the main queue waits (round 6): from a rocprofv3 kernel trace of the bench, over the last STEPS steps (step
boundaries as tools/prof_summary.py), every main-queue idle gap above 5 us, grouped by the (previous, next) main
kernel pair, with the share of the gap during which another queue had a kernel running (a cross-stream wait shows as
a gap the side queue fills).  Usage: stream_gaps.py TRACE.csv [STEPS]."""
import collections
import csv
import sys


def short(k):
    return k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:48]


path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "gen_aligner_in" in r["Kernel_Name"]]
sel = rows[starts[-steps]:]
qk = collections.Counter(r.get("Queue_Id", "0") for r in sel)
mq = qk.most_common(1)[0][0]
main = [r for r in sel if r.get("Queue_Id", "0") == mq]
other = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"])) for r in sel
                if r.get("Queue_Id", "0") != mq))
agg = collections.defaultdict(lambda: [0, 0.0, 0.0, collections.Counter()])
total = 0.0
for a, b in zip(main, main[1:]):
    g0, g1 = int(a["End_Timestamp"]), int(b["Start_Timestamp"])
    if g1 - g0 <= 5000:
        continue
    cov = 0
    for s, e, k in other:
        if e <= g0:
            continue
        if s >= g1:
            break
        ov = min(e, g1) - max(s, g0)
        if ov > 0:
            cov += ov
            agg[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))][3][k] += ov
    key = (short(a["Kernel_Name"]), short(b["Kernel_Name"]))
    agg[key][0] += 1
    agg[key][1] += (g1 - g0) / 1e3
    agg[key][2] += cov / 1e3
    total += (g1 - g0) / 1e3
print(f"main queue {mq}: gaps > 5 us total {total / steps:.1f} us/step over {steps} steps")
for (pa, nb), (n, us, cov, ks) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:20]:
    top = ", ".join(f"{k} {v / 1e3 / steps:.0f}" for k, v in ks.most_common(2))
    print(f"{us / steps:8.1f} us/step {n // steps:3d}/step  other queue busy {cov / max(us, 1e-9):4.0%}  "
          f"{pa} -> {nb}   [{top}]")
