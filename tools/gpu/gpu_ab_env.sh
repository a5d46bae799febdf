# same-box alternating A/B of one ablation-build env knob on the step bench (ABENV="NAME=VALUE")
set -o pipefail
mkdir -p gpurun_out/ab_env
export TMPDIR=/tmp
export OSPO_HIP_LIB=$PWD/ospo_amd/libospo_hip_ablation.so
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_env/a$i.json 2>/dev/null || { echo "A FAILED"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_env/a$i.json')); print('A', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
  env $ABENV timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab_env/b$i.json 2>/dev/null || { echo "B FAILED"; exit 1; }
  python -c "import json; d=json.load(open('gpurun_out/ab_env/b$i.json')); print('B', d['value'], d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
env $ABENV timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/ab_env/prof -o prof -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > /dev/null 2>&1 || { echo "PROF FAILED"; exit 1; }
python tools/prof_summary.py gpurun_out/ab_env/prof/prof_kernel_trace.csv 5 25
