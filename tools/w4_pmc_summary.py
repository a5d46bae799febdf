"""Per-launch counter means per kernel from tools/gpu/gpu_r04_w4_pmc.sh (FETCH_SIZE doubled for 16-B/lane
streaming reads, MI355X_MICROARCH.md HBM; effective clock = GRBM_GUI_ACTIVE / 8 XCDs / kernel time)."""
import collections
import csv
import glob
import json
import sys

src = sys.argv[1]
acc = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for f in glob.glob(f"{src}/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        name = ("w4" if "gemm_nt_w4_kernel" in k else "sp8" if "gemm_nt_v5_kernel" in k else
                "hipblaslt" if "Cijk" in k else "fixup" if "splitk_fixup" in k else None)
        if name is None:
            continue
        acc[name][r["Counter_Name"]].append(float(r["Counter_Value"]))
        if "End_Timestamp" in r and "Start_Timestamp" in r:
            dur[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) * 1e-3)
out = {}
for name, cs in acc.items():
    m = {c: sum(v) / len(v) for c, v in cs.items()}
    d = {"launches_per_pass": len(next(iter(cs.values())))}
    if "FETCH_SIZE" in m:
        d["fetch_bytes"] = round(2 * m["FETCH_SIZE"] * 1024)
    if "WRITE_SIZE" in m:
        d["write_bytes"] = round(m["WRITE_SIZE"] * 1024)
    if "TCC_HIT_sum" in m:
        d["l2_hit_rate"] = round(m["TCC_HIT_sum"] / (m["TCC_HIT_sum"] + m["TCC_MISS_sum"]), 4)
    if "SQ_VALU_MFMA_BUSY_CYCLES" in m and "SQ_BUSY_CYCLES" in m:
        d["mfma_busy_per_busy"] = round(m["SQ_VALU_MFMA_BUSY_CYCLES"] / (m["SQ_BUSY_CYCLES"] * 4 * 1024 / 32), 4)
    if dur[name]:
        t = sorted(dur[name])[len(dur[name]) // 2]
        d["us_median"] = round(t, 1)
        if "GRBM_GUI_ACTIVE" in m:
            d["eff_clock_ghz"] = round(m["GRBM_GUI_ACTIVE"] / 8 / t / 1e3, 3)
    for c in ("SQ_INSTS_LDS", "SQ_LDS_BANK_CONFLICT", "SQ_LDS_IDX_ACTIVE", "SQ_WAVE_CYCLES", "SQ_WAIT_ANY",
              "SQ_BUSY_CYCLES", "SQ_VALU_MFMA_BUSY_CYCLES", "GRBM_GUI_ACTIVE"):
        if c in m:
            d[c] = round(m[c])
    out[name] = d
print(json.dumps(out, indent=1))
