# Round 5: T2I bench with the VQ pixel decode pipelined on a side stream (default) vs serial, 2 alternating rounds;
# tokens and pixels checksums must agree
# (ran against the bench.py of that experiment, which had --t2i-serial-decode and a pipelined default; the bench keeps the serial step)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5tq}
for i in 1 2; do
  for V in pipe serial; do
    A=""; [ $V = serial ] && A="--t2i-serial-decode"
    timeout -k 10 300 python -u bench.py --workload t2i --steps 3 --warmup 1 --no-cpu-baseline $A > gpurun_out/${TAG}_${V}_${i}.json 2> gpurun_out/${TAG}_${V}_${i}.err || { echo "T2I $V FAILED"; tail -20 gpurun_out/${TAG}_${V}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['avg_step_us'], d['tokens_checksum'], d['pixels_checksum'], d['config']['vq_decode_ms_per_batch'])" gpurun_out/${TAG}_${V}_${i}.json $V
  done
done
