# Round 5 call D: side-stream price, rocprof breakdown of the current default, GEMM counter traffic of the 8-pair
# and MXFP8 lines
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
bash tools/gpu/gpu_r05_side.sh || exit 1
TAG=r5p bash tools/gpu/gpu_r05_prof.sh || exit 1
bash tools/gpu/gpu_r05_pmc.sh || exit 1
