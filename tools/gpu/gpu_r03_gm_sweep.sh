# GEMM L2 row-group size (GM 4 default; variants 20/21/22 = GM 2/8/16) per step shape, interleaved rounds (+ RoPE qkv)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GB_VARIANTS=0,20,21,22 GB_ROPE=1 timeout -k 10 500 python -u tools/gemm_bench.py > gpurun_out/gm_sweep_r3.jsonl 2> gpurun_out/gm_sweep_r3.err || { echo "GEMM BENCH FAILED"; tail -5 gpurun_out/gm_sweep_r3.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/gm_sweep_r3.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    print(d["shape"], {k: round(d[k]["ms"] * 1e3, 1) for k in ("v0", "v20", "v21", "v22") if k in d}, d.get("bit_equal_v0"))
PY
