# Round 5: GEMM counter traffic (2*FETCH_SIZE + WRITE_SIZE per launch) of the 8-pair line (config 3's per-GPU
# batch) and of the MXFP8 r = 32 line (config 5), each in its own counter passes (tools/gpu/gpu_pmc_bench.sh)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
PMC_DIR=gpurun_out/pmc_p8 BENCH_ARGS="--pairs-per-gpu 8" bash tools/gpu/gpu_pmc_bench.sh || exit 1
BENCH_ARGS="--pairs-per-gpu 8" python tools/pmc_summary.py gpurun_out/pmc_p8 gpurun_out/gemm_pmc_bf16_p8_r16_l30.json > /dev/null || exit 1
PMC_DIR=gpurun_out/pmc_mx8 BENCH_ARGS="--linear-dtype mx8 --lora-r 32" bash tools/gpu/gpu_pmc_bench.sh || exit 1
BENCH_ARGS="--linear-dtype mx8 --lora-r 32" python tools/pmc_summary.py gpurun_out/pmc_mx8 gpurun_out/gemm_pmc_mx8_p4_r32_l30.json > /dev/null || exit 1
head -c 600 gpurun_out/gemm_pmc_bf16_p8_r16_l30.json; echo; head -c 600 gpurun_out/gemm_pmc_mx8_p4_r32_l30.json; echo
rm -rf gpurun_out/pmc_p8 gpurun_out/pmc_mx8
