# Round 5: price of the LoRA weight-gradient side stream on the current tree (ABL=grads removes it; results invalid),
# same box, alternating with the default step
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5j}
for i in 1 2; do
  for V in default nograds; do
    if [ $V = default ]; then CMD="python -u bench.py"; else CMD="python -u tools/ablate_side.py"; fi
    ABL=grads timeout -k 10 300 $CMD --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper \
      > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err \
      || { echo "BENCH $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
