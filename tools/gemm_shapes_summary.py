"""Per-shape GEMM time from a rocprofv3 kernel trace of the bench (round 5).

The GEMM launches of a step come in a fixed order, so the i-th `gemm_nt_*` launch of every timed step is
the same shape.  Launches are grouped by (grid, the split-K fixup that follows on the same queue) and
printed with their count per step and the average duration over the last STEPS steps (step boundaries as
in prof_summary.py: the aligner-input gather that opens every step).

usage: python tools/gemm_shapes_summary.py <kernel_trace.csv> [STEPS]
"""
import collections
import csv
import sys

path = sys.argv[1]
steps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
rows = list(csv.DictReader(open(path)))
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
starts = [i for i, r in enumerate(rows) if "gen_aligner_in" in r["Kernel_Name"]]
sel = rows[starts[-steps]:]


def dur(r):
    return (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3


def grid(r):
    return tuple(int(r.get(f"Grid_Size_{a}", 0) or 0) for a in "XYZ")


groups = collections.OrderedDict()
last_gemm = {}
for r in sel:
    name = r["Kernel_Name"]
    q = r.get("Queue_Id", "0")
    if "gemm_nt" in name and "fixup" not in name:
        key = ("gemm", grid(r))
        g = groups.setdefault(key, [0, 0.0, 0, 0.0])
        g[0] += 1
        g[1] += dur(r)
        last_gemm[q] = key
    elif "splitk_fixup" in name and q in last_gemm:
        g = groups[last_gemm.pop(q)]
        g[2] += 1
        g[3] += dur(r)
tot = 0.0
print(f"{'grid':>22} {'per step':>8} {'gemm us':>9} {'fixups':>7} {'fixup us':>9} {'ms/step':>8}")
for (kind, gr), (n, t, nf, tf) in sorted(groups.items(), key=lambda kv: -(kv[1][1] + kv[1][3])):
    ms = (t + tf) / 1e3 / steps
    tot += ms
    print(f"{str(gr):>22} {n / steps:8.1f} {t / n:9.1f} {nf / steps:7.1f} {(tf / nf if nf else 0):9.1f} {ms:8.2f}")
print(f"total GEMM + fixup {tot:.2f} ms/step")
