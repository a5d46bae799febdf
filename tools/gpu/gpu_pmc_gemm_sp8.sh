# PMC passes of the SP8 GEMM (qkv_fwd shape, 10 launches): LDS conflicts / instruction mix / MFMA busy
set -o pipefail
mkdir -p gpurun_out/pmc_sp8
export TMPDIR=/tmp
export GO_VARIANT=0 GO_ITERS=10
timeout -s KILL 90 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_sp8/a -o p -- python tools/gemm_one.py > /dev/null 2>> gpurun_out/pmc_sp8/err.log || { echo "pass a failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc_sp8/b -o p -- python tools/gemm_one.py > /dev/null 2>> gpurun_out/pmc_sp8/err.log || { echo "pass b failed"; exit 1; }
timeout -s KILL 90 rocprofv3 --pmc SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA SQ_INSTS_VALU GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d gpurun_out/pmc_sp8/c -o p -- python tools/gemm_one.py > /dev/null 2>> gpurun_out/pmc_sp8/err.log || { echo "pass c failed"; exit 1; }
python - <<'PY'
import csv, glob, json, collections
tot = collections.defaultdict(float); n = collections.Counter()
for f in glob.glob("gpurun_out/pmc_sp8/*/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        if "gemm_nt_v5_kernel" not in r["Kernel_Name"]:
            continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n[r["Counter_Name"]] += 1
out = {k: tot[k] / max(1, len({1})) for k in tot}
print(json.dumps({k: round(v) for k, v in sorted(out.items())}))
PY
