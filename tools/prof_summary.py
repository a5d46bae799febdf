"""Per-step kernel breakdown from a rocprofv3 kernel trace: uses the last STEPS
occurrences of the step's first kernel (the aligner-input gather) as step
boundaries, so one-time setup (weight init / transposes) is excluded."""
import csv
import collections
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "gen_aligner_in" in r["Kernel_Name"]]
first = starts[-steps]
sel = rows[first:]
t0, t1 = int(sel[0]["Start_Timestamp"]), max(int(r["End_Timestamp"]) for r in sel)
agg = collections.defaultdict(lambda: [0, 0.0])
for r in sel:
    k = r["Kernel_Name"]
    k = k.replace("void ", "").replace("(anonymous namespace)::", "")
    k = k.split("(")[0][:70]
    agg[k][0] += 1
    agg[k][1] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6
busy = sum(v[1] for v in agg.values())
print(f"wall {((t1 - t0) / 1e6) / steps:.2f} ms/step, kernel-sum {busy / steps:.2f} ms/step")
# main queue (the one with the most kernels): its kernel-time sum, and the idle gaps between its kernels
qk = collections.Counter(r.get("Queue_Id", "0") for r in sel)
mq = qk.most_common(1)[0][0]
main = [r for r in sel if r.get("Queue_Id", "0") == mq]
mbusy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in main) / 1e6
gaps = [int(b["Start_Timestamp"]) - int(a["End_Timestamp"]) for a, b in zip(main, main[1:])]
pos = [g for g in gaps if g > 0]
print(f"main queue {mq}: {len(main) // steps} kernels/step, busy {mbusy / steps:.2f} ms/step, idle gaps "
      f"{sum(pos) / 1e6 / steps:.2f} ms/step (median gap {sorted(pos)[len(pos) // 2] / 1e3 if pos else 0:.1f} us)")
for k, (n, ms) in sorted(agg.items(), key=lambda kv: -kv[1][1])[:int(sys.argv[3]) if len(sys.argv) > 3 else 30]:
    print(f"{ms / steps:8.2f} ms/step {n // steps:5d}/step {ms / n * 1e3:9.1f} us  {k}")
