# HBM-side traffic of the attention kernels (FETCH_SIZE / WRITE_SIZE / TCC hit-miss), block-major vs group-major order
set -o pipefail
mkdir -p gpurun_out/attn_tr
export TMPDIR=/tmp
for ORD in 0 1; do
  for SET in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    tag=$(echo $SET | cut -d' ' -f1)_o$ORD
    OSPO_ATTN_ORDER=$ORD timeout -s KILL 120 rocprofv3 --pmc $SET --output-format csv -d gpurun_out/attn_tr/$tag -o p -- python tools/attn_bench.py > gpurun_out/attn_tr/$tag.log 2>&1 || { echo "PMC $tag FAILED"; tail -3 gpurun_out/attn_tr/$tag.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, collections
for f in sorted(glob.glob("gpurun_out/attn_tr/*/p_counter_collection.csv")):
    agg = collections.defaultdict(float); n = collections.Counter(); seen=set()
    for r in csv.DictReader(open(f)):
        k = r["Kernel_Name"].split("(")[0].replace("void ", "").replace("(anonymous namespace)::", "")[-40:]
        if "attn_bwd" not in k: continue
        agg[(k, r["Counter_Name"])] += float(r["Counter_Value"])
        if (k, r["Dispatch_Id"]) not in seen: seen.add((k, r["Dispatch_Id"])); n[k] += 1
    for (k, c), v in sorted(agg.items()):
        print(f.split("/")[-2], k, c, f"{v / n[k]:.4g}")
PY
