# attention tests + backward A/B (env ABVAR=NAME selects the B side in the ablation build) + per-kernel stats
set -o pipefail
mkdir -p gpurun_out/attn_ab
export TMPDIR=/tmp
ABVAR=${ABVAR:-OSPO_ATTN_DQ_2SLOT}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k "flash" -m gpu > gpurun_out/attn_ab/tests.log 2>&1 || { echo "TESTS FAILED"; grep -E "^FAILED|Error" gpurun_out/attn_ab/tests.log | head; tail -3 gpurun_out/attn_ab/tests.log; exit 1; }
tail -1 gpurun_out/attn_ab/tests.log
for i in 1 2; do
  timeout -k 10 120 python tools/attn_bench.py 2>/dev/null || { echo "FAILED A"; exit 1; }
  env $ABVAR=1 timeout -k 10 120 python tools/attn_bench.py 2>/dev/null || { echo "FAILED B"; exit 1; }
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/attn_ab/prof -o p -- python tools/attn_bench.py > gpurun_out/attn_ab/prof.log 2>&1 || { echo "PROF FAILED"; exit 1; }
python - <<'PY'
import csv, glob
f = glob.glob("gpurun_out/attn_ab/prof/*kernel_stats.csv")[0]
for r in csv.DictReader(open(f)):
    if "attn" in r["Name"]:
        print(f'{float(r["AverageNs"])/1e3:8.1f} us  x{r["Calls"]:>4}  {r["Name"][:80]}')
PY
