"""Per-decode-step kernel breakdown of tools/t2i_prof.py's trace: the last STEPS decode steps
(one advance_kernel per step)."""
import collections
import csv
import sys

rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda r: int(r["Start_Timestamp"]))
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ends = [i for i, r in enumerate(rows) if "advance_kernel" in r["Kernel_Name"]]
sel = rows[ends[-steps - 1] + 1: ends[-1] + 1]
t0, t1 = int(sel[0]["Start_Timestamp"]), int(sel[-1]["End_Timestamp"])
agg = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    k = r["Kernel_Name"].replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0][:60]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
busy = sum(v[1] for v in agg.values())
print(f"wall {(t1 - t0) / 1e3 / steps:.1f} us/step (eager), kernel-sum {busy / steps:.1f} us/step")
for k, (n, us) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print(f"{us / steps:9.1f} us/step {n // steps:4d}/step {us / n:8.1f} us  {k}")
