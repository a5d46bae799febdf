# A/B of NT GEMM schedules on the step shapes (ablation build), same process
set -o pipefail
mkdir -p gpurun_out
GB_VARIANTS=${GB_VARIANTS:-0,24,25} timeout -k 10 500 python tools/gemm_bench.py > gpurun_out/gemm_ab.jsonl 2> gpurun_out/gemm_ab.err
