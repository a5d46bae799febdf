# Round 6: HBM bytes per forward-attention launch by workgroup-order band size (FETCH_SIZE and WRITE_SIZE passes)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
D=gpurun_out/attn_pmc
mkdir -p $D
for GM in default 8 4 32; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $D/${GM}_$C -o p -- python tools/attn_fwd_pmc.py $GM > $D/${GM}_$C.log 2>&1 || { echo "pass $GM $C failed"; tail -5 $D/${GM}_$C.log; exit 1; }
  done
done
python - <<'PY'
import csv, glob, collections, json
out = {}
for gm in ("default", "8", "4", "32"):
    tot = {}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        f = glob.glob(f"gpurun_out/attn_pmc/{gm}_{c}/**/*counter_collection.csv", recursive=True)[0]
        v, n = 0.0, 0
        for r in csv.DictReader(open(f)):
            if "attn_fwd3" in r["Kernel_Name"]:
                v += float(r["Counter_Value"]); n += 1
        tot[c] = v / max(n, 1)
    mib = (2 * tot["FETCH_SIZE"] + tot["WRITE_SIZE"]) / 1024
    out[gm] = {"MiB_per_launch": round(mib, 1), "x_algorithmic": round(mib / 150.6, 3)}
print(json.dumps({"attn_fwd3_hbm_by_band (2 x FETCH_SIZE + WRITE_SIZE; algorithmic 150.6 MiB: Q K V read once, O + lse written)": out}))
PY
find $D -name "*counter_collection.csv" -delete
