# Round 5, verdict r4 item 3c: plain-epilogue store variants of the w4 GEMM (ablation library), same process
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5f}
timeout -k 10 400 python -u tools/gemm_epi_ab.py > gpurun_out/${TAG}_gemm_epi.log 2>&1 || { echo "EPI AB FAILED"; tail -20 gpurun_out/${TAG}_gemm_epi.log; exit 1; }
cut -c1-300 gpurun_out/${TAG}_gemm_epi.log
