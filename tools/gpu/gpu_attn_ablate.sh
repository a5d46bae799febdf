# attention backward decomposition (ablation build, results invalid by design for DBG != 0)
set -o pipefail
mkdir -p gpurun_out
for v in 0 5 1 2 3 4; do
  OSPO_ATTN_DKDV_DBG=$v timeout -k 10 120 python tools/attn_bench.py > gpurun_out/attn_dbg$v.json 2>/dev/null || { echo "FAILED $v"; exit 1; }
  echo "dbg=$v $(cat gpurun_out/attn_dbg$v.json)"
done
