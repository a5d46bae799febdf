"""Per-launch HBM bytes and MFMA busy of the bench's kernels from tools/gpu/gpu_pmc_bench.sh.

HBM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE (MI355X_MICROARCH.md: on gfx950
FETCH_SIZE reports half the bytes of 16-B/lane streaming reads; WRITE_SIZE is exact),
FETCH/WRITE_SIZE in KiB.  The NT GEMM's split-K fixup launches are charged to the GEMM
(the bench times them inside the same launch window).  Writes profiles/gemm_pmc.json, or the file named by
the second argument (round 5: one file per bench configuration, bench.gemm_pmc_path)."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "pmc_bench")
dst = sys.argv[2] if len(sys.argv) > 2 else os.path.join(ROOT, "profiles", "gemm_pmc.json")


def load(tag):
    f = max(glob.glob(os.path.join(src, tag, "**", "*counter_collection.csv"), recursive=True), key=os.path.getmtime)
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        per[k][r["Counter_Name"]] += float(r["Counter_Value"])
        n[(k, r["Counter_Name"])] += 1
    return per, n


def short(k):
    return k.replace("void ", "").replace("(anonymous namespace)::", "").split("(")[0]


fetch, nf = load("FETCH_SIZE")
write, nw = load("WRITE_SIZE")
sq, ns = load("SQ_VALU_MFMA_BUSY_CYCLES")
out = {}
GEMM_NAMES = ("gemm_nt_w4_kernel", "gemm_nt_v5_kernel")  # round 4 default / the SP8 schedule


def is_mx(k):
    """MXFP8 main operands: gemm_nt_v5_kernel<DBG, DROP, MX, SP> / gemm_nt_w4_kernel<DROP, DBG, V, MX>."""
    args = [a.strip() for a in k.split("<", 1)[1].split(">", 1)[0].split(",")] if "<" in k else []
    pos = 2 if "gemm_nt_v5_kernel" in k else 3
    return len(args) > pos and args[pos] == "true"


gemm_all = [k for k in fetch if any(g in k for g in GEMM_NAMES)]
fix = [k for k in fetch if "splitk_fixup" in k]
# kernel wall time of the same dispatches (counter rows carry the dispatch timestamps)
f = glob.glob(os.path.join(src, "SQ_VALU_MFMA_BUSY_CYCLES", "**", "*counter_collection.csv"), recursive=True)[0]
durs = collections.defaultdict(dict)
for r in csv.DictReader(open(f)):
    if any(g in r["Kernel_Name"] for g in GEMM_NAMES):
        durs[is_mx(r["Kernel_Name"])][r["Dispatch_Id"]] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
fams = {False: [k for k in gemm_all if not is_mx(k)], True: [k for k in gemm_all if is_mx(k)]}
fams = {m: ks for m, ks in fams.items() if ks}
# the split-K fixups go with the family that launches most GEMMs (the bench times them inside its launches)
main_fam = max(fams, key=lambda m: sum(nf[(k, "FETCH_SIZE")] for k in fams[m]))
for m, ks in fams.items():
    launches = sum(nf[(k, "FETCH_SIZE")] for k in ks)
    kib = sum(2 * fetch[k]["FETCH_SIZE"] + write[k]["WRITE_SIZE"] for k in ks + (fix if m == main_fam else []))
    busy = sum(sq[k]["SQ_VALU_MFMA_BUSY_CYCLES"] for k in sq if k in ks)
    dur_s = sum(durs[m].values()) * 1e-9
    out["gemm_nt_mx8_256x256" if m else "gemm_nt_256x256"] = {
        "hbm_bytes_per_launch": round(kib * 1024 / launches),
        "launches": int(launches),
        "kernels": sorted({short(k) for k in ks}),
        "method": "2*FETCH_SIZE + WRITE_SIZE (KiB), the NT GEMM" + (" + splitk_fixup_kernel" if m == main_fam else "")
                  + ", averaged over launches",
        # SQ_VALU_MFMA_BUSY_CYCLES: summed over the 1024 SIMDs, against the cycles of the counter pass's kernel
        # durations at the 2.4 GHz peak clock.  (The round-3 clock from GRBM_GUI_ACTIVE / 8 / duration came out
        # above 2.4 GHz and is no longer reported; in-kernel clocks come from s_memtime / s_memrealtime stamps,
        # tools/w4_stamps.py.)
        "mfma_busy_frac_at_2p4ghz_peak": round(busy / (dur_s * 2.4e9 * 1024), 4) if dur_s else None,
    }
ranked = sorted(set(fetch) | set(write), key=lambda k: -(2 * fetch[k]["FETCH_SIZE"] + write[k]["WRITE_SIZE"]))
for k in ranked[:15] + [k for k in ranked[15:] if "attn" in k]:  # (round 6: every attention kernel)
    n = max(nf[(k, "FETCH_SIZE")], 1)
    out.setdefault("per_kernel_MiB_per_launch", {})[short(k)[:60]] = round(
        (2 * fetch[k]["FETCH_SIZE"] + write[k]["WRITE_SIZE"]) / 1024 / n, 2)
out["bench_args"] = os.environ.get("BENCH_ARGS", "")
json.dump(out, open(dst, "w"), indent=1)
print(json.dumps(out, indent=1))
