# Round 5: same-box step A/B of the round-5 kernel changes, alternating, default bench workload (4 pairs):
#   base  = libospo_hip_r5nostage.so (round-5 hash, round-4 GEMM stores / attention order / forward rescale)
#   nont  = libospo_hip_r5nont.so    (the product tree with plain GEMM output stores)
#   new   = the product library      (non-temporal GEMM output stores, banded attention-backward order, O rescale
#                                     only when a running max moved)
#   gdbgu = the product library with --lora-variant gdb_gu_only (q|k|v, o, down: skinny g + side-stream dB)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5i}
for i in 1 2; do
  for V in base nont new gdbgu; do
    A=""
    case $V in
      base) export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_r5nostage.so ;;
      nont) export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_r5nont.so ;;
      new) unset OSPO_HIP_LIB ;;
      gdbgu) unset OSPO_HIP_LIB; A="--lora-variant gdb_gu_only" ;;
    esac
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper $A \
      > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err \
      || { echo "BENCH $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'], d['loss_first_step'])" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
unset OSPO_HIP_LIB
