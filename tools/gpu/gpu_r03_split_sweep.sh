# Split-K tail: the cost model's choice (v0) against every pinned split, per step shape, interleaved rounds
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
GB_VARIANTS=0 GB_SPLITS=1,2,3,4,5,6,8 timeout -k 10 500 python -u tools/gemm_bench.py > gpurun_out/split_sweep_r3.jsonl 2> gpurun_out/split_sweep_r3.err || { echo "GEMM BENCH FAILED"; tail -5 gpurun_out/split_sweep_r3.err; exit 1; }
python - <<'PY'
import json
for l in open("gpurun_out/split_sweep_r3.jsonl"):
    if not l.startswith("{"): continue
    d = json.loads(l)
    print(d["shape"], {k: round(d[k]["ms"] * 1e3, 1) for k in d if k.startswith("v0") or k.startswith("split")})
PY
