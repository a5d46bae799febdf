"""Per-kernel counters of the bench step (tools/gpu/gpu_pmc_bench.sh passes) -> profiles/r03/pmc_step.json.

For every kernel of the step: launches, average duration (the counter rows' dispatch timestamps of the
SQ pass), HBM-side bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: gfx950
FETCH_SIZE reports half of 16-B/lane streaming reads; WRITE_SIZE is exact; both include Infinity-Cache
hits), the resulting GB/s, and MFMA busy = SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE / 8 x 1024 SIMDs)
with the effective clock GRBM_GUI_ACTIVE / 8 / duration.  Counter passes run slower than un-profiled
launches (DVFS, MI355X_MICROARCH.md give-back item 2): durations here are for the ratios, not timing.

python tools/pmc_step.py [gpurun_out/pmc_bench] [out.json]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_bench")
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "r03", "pmc_step.json")


def short(k):
    return k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


def load(tag):
    f = max(glob.glob(os.path.join(src, tag, "**", "*counter_collection.csv"), recursive=True), key=os.path.getmtime)
    vals = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(dict)
    for r in csv.DictReader(open(f)):
        k = short(r["Kernel_Name"])
        vals[k][r["Counter_Name"]] += float(r["Counter_Value"])
        disp[k][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return vals, disp


fetch, fd = load("FETCH_SIZE")
write, _ = load("WRITE_SIZE")
sq, sd = load("SQ_VALU_MFMA_BUSY_CYCLES")
out = {}
for k in sorted(set(fetch) | set(sq), key=lambda k: -sum(sd.get(k, fd.get(k, {})).values())):
    n = len(fd.get(k, {})) or len(sd.get(k, {}))
    if not n:
        continue
    dur = sum(sd[k].values()) / max(len(sd[k]), 1) * 1e-9 if sd.get(k) else None
    nbytes = (2 * fetch[k]["FETCH_SIZE"] + write[k]["WRITE_SIZE"]) * 1024 / n
    gui = sq[k].get("GRBM_GUI_ACTIVE", 0.0)
    busy = sq[k].get("SQ_VALU_MFMA_BUSY_CYCLES", 0.0)
    tot_dur = sum(sd[k].values()) * 1e-9 if sd.get(k) else None
    out[k[:90]] = {
        "launches": n,
        "avg_us_profiled": round(dur * 1e6, 2) if dur else None,
        "hbm_bytes_per_launch": round(nbytes),
        "read_bytes_per_launch": round(2 * fetch[k]["FETCH_SIZE"] * 1024 / n),
        "write_bytes_per_launch": round(write[k]["WRITE_SIZE"] * 1024 / n),
        "GBps_profiled": round(nbytes / dur / 1e9, 1) if dur else None,
        "mfma_busy_frac_of_active_cycles": round(busy / (gui / 8 * 1024), 4) if gui else None,
        "effective_clock_ghz": round(gui / 8 / tot_dur / 1e9, 3) if gui and tot_dur else None,
    }
os.makedirs(os.path.dirname(dst), exist_ok=True)
json.dump({"method": __doc__.split("\n\n")[1].replace("\n", " "), "kernels": out}, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1)[:6000])
