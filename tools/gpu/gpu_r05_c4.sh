# Round 5, call C4: GEMM / per-kernel counter traffic of the product tree (plain GEMM stores) at the default
# 4-pair line (-> profiles/gemm_pmc.json), the 8-pair line and the MXFP8 r = 32 line (gpu_r05_pmc.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PMC_DIR=gpurun_out/pmc_p4 BENCH_ARGS="" bash tools/gpu/gpu_pmc_bench.sh || exit 1
BENCH_ARGS="" python tools/pmc_summary.py gpurun_out/pmc_p4 gpurun_out/gemm_pmc.json > /dev/null || exit 1
head -c 600 gpurun_out/gemm_pmc.json; echo
rm -rf gpurun_out/pmc_p4
bash tools/gpu/gpu_r05_pmc.sh
