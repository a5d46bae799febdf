# Round 5, verdict r4 item 4: the fused g / dB stream for every group (default) against gdb_gu_only (q|k|v, o, down:
# g from the skinny product on the main stream, dB on the side stream), same box, alternating
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5g}
for i in 1 2; do
  for V in default gdb_gu_only; do
    A=""; [ $V != default ] && A="--lora-variant $V"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper $A \
      > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err \
      || { echo "BENCH $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
