# Round 5: the LoRA dA side stream vs running groups of it on the main stream (bench --lora-variant main_<group>),
# default workload, 2 alternating rounds on one box
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
TAG=${TAG:-r5side}
for i in 1 2; do
  for V in base main_qkv,main_o,main_gu,main_down main_down main_qkv,main_o,main_gu; do
    N=$(echo $V | tr ',' '-')
    A=""; [ $V != base ] && A="--lora-variant $V"
    timeout -k 10 300 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-wrapper $A > gpurun_out/${TAG}_${N}_${i}.json 2> gpurun_out/${TAG}_${N}_${i}.err || { echo "BENCH $V FAILED"; tail -20 gpurun_out/${TAG}_${N}_${i}.err; exit 1; }
    python -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('loss_first_step'))" gpurun_out/${TAG}_${N}_${i}.json $N
  done
done
