"""Measured vs algorithmic HBM bytes of the T2I decode kernels from tools/gpu/gpu_r04_t2i_pmc.sh's counter passes.

Decode kernels: dlin_kernel (every decode Linear, incl. gen_head / aligner), attn_cache2_kernel, cfg_sample, the
aligner input kernel, advance.  Their measured bytes (2 x FETCH_SIZE + WRITE_SIZE, MI355X_MICROARCH.md's gfx950
correction; KiB counters) over the whole eager generate() of tools/t2i_pmc.py are compared with the algorithmic
bytes of the same work: bench.t2i_bytes_per_step for each of the N - 1 decode steps (KV cache of positions
Lp .. Lp + s) plus the prefill's head (gen_head + aligner weights, once).  Writes profiles/t2i_pmc.json with
the ratio; bench.py --workload t2i reports roofline.traffic = ratio x its own algorithmic bytes per step."""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402
from ospo_amd.engine import JANUS_PRO_7B  # noqa: E402

DECODE = ("dlin_kernel", "attn_cache2_kernel", "cfg_sample_kernel", "gen_aligner_in8_kernel", "advance_kernel")


def load(src, tag):
    f = max(glob.glob(os.path.join(src, tag, "**", "*counter_collection.csv"), recursive=True), key=os.path.getmtime)
    per = collections.defaultdict(float)
    n = collections.Counter()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"]
        name = next((d for d in DECODE if d in k), None)
        if name is None:
            continue
        per[name] += float(r["Counter_Value"]) * 1024.0
        n[name] += 1
    return per, n


def main():
    src = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "gpurun_out", "t2i_pmc")
    n_img, lp, rows = int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    fetch, nf = load(src, "FETCH_SIZE")
    write, nw = load(src, "WRITE_SIZE")
    dims = JANUS_PRO_7B
    D, Dg, V = dims.d_model, dims.gen_head_dim, dims.img_vocab
    head = 2.0 * (D * Dg + Dg * V + D * D)
    alg = head + sum(bench.t2i_bytes_per_step(dims, rows, lp + s) for s in range(1, n_img))
    measured = sum(2 * fetch[k] + write[k] for k in fetch)
    per_kernel = {k: {"dispatches": nf[k], "fetch_bytes_x2": round(2 * fetch[k]), "write_bytes": round(write[k])}
                  for k in sorted(fetch)}
    out = {"source": "tools/gpu/gpu_r04_t2i_pmc.sh (rocprofv3 --pmc FETCH_SIZE, then WRITE_SIZE; eager generate)",
           "n_img_tokens": n_img, "prompt_len": lp, "rows": rows, "decode_steps": n_img - 1,
           "measured_bytes": round(measured), "algorithmic_bytes": round(alg),
           "traffic_ratio": round(measured / alg, 4), "per_kernel": per_kernel}
    json.dump(out, open(os.path.join(ROOT, "profiles", "t2i_pmc.json"), "w"), indent=1)
    print(json.dumps({k: out[k] for k in ("measured_bytes", "algorithmic_bytes", "traffic_ratio")}))


if __name__ == "__main__":
    main()
