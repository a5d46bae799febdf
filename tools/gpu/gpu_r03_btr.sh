# skinny3 with register Bt fragments (OSPO_SK3_BTREG): bit-for-bit check against the staged form, then timings
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
timeout -k 10 120 python -u tools/skinny_btr_check.py gpurun_out/btr_off.pt > gpurun_out/btr_check.log 2>&1 || { echo "CHECK off FAILED"; tail -5 gpurun_out/btr_check.log; exit 1; }
OSPO_SK3_BTREG=1 timeout -k 10 120 python -u tools/skinny_btr_check.py gpurun_out/btr_on.pt >> gpurun_out/btr_check.log 2>&1 || { echo "CHECK on FAILED"; tail -5 gpurun_out/btr_check.log; exit 1; }
python tools/skinny_btr_check.py --compare gpurun_out/btr_off.pt gpurun_out/btr_on.pt || { echo "BTR NOT BIT-IDENTICAL"; exit 1; }
rm -f gpurun_out/btr_*.pt
for v in off on; do
  if [ $v = on ]; then export OSPO_SK3_BTREG=1; else unset OSPO_SK3_BTREG; fi
  echo "BTREG=$v"; timeout -k 10 120 python -u tools/skinny_diag.py 2>&1 | grep -v amdgpu.ids || exit 1
done
