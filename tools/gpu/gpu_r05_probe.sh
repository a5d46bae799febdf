# Round 5, verdict r4 items 3a / 3b / 5: the fixed MFMA clock probe (one run, HIP errors checked, random and
# zero operands), the w4 GEMM's in-kernel clock on random vs zero operands (ablation stamps), and the
# trajectory test's step-1 bf16-vs-fp32 oracle gap dissected (tools/traj_diag.py).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5b}
timeout -k 10 120 ./tools/mfma_clock_probe > gpurun_out/${TAG}_mfma_clock.log 2>&1 || { echo "PROBE FAILED rc=$?"; cat gpurun_out/${TAG}_mfma_clock.log; exit 1; }
cat gpurun_out/${TAG}_mfma_clock.log
timeout -k 10 180 python -u tools/w4_stamps.py > gpurun_out/${TAG}_w4_stamps_random.log 2>&1 || { echo "STAMPS FAILED"; tail gpurun_out/${TAG}_w4_stamps_random.log; exit 1; }
W4_DATA=zero timeout -k 10 180 python -u tools/w4_stamps.py > gpurun_out/${TAG}_w4_stamps_zero.log 2>&1 || { echo "STAMPS0 FAILED"; tail gpurun_out/${TAG}_w4_stamps_zero.log; exit 1; }
cut -c1-330 gpurun_out/${TAG}_w4_stamps_random.log gpurun_out/${TAG}_w4_stamps_zero.log
timeout -k 10 600 python -u tools/traj_diag.py > gpurun_out/${TAG}_traj_diag.log 2>&1 || { echo "TRAJ FAILED"; tail -20 gpurun_out/${TAG}_traj_diag.log; exit 1; }
cut -c1-1500 gpurun_out/${TAG}_traj_diag.log
