# side-stream / skinny ablations against the default step, alternating, same box (results invalid)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for r in 1 2; do
  for A in none grads skinny; do
    if [ $A = none ]; then
      timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl_${A}_$r.json 2>/dev/null || exit 1
    else
      ABL=$A timeout -k 10 300 python tools/ablate_side.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/abl_${A}_$r.json 2>/dev/null || exit 1
    fi
    python -c "import json; d=json.load(open('gpurun_out/abl_${A}_$r.json')); print('$A', $r, d['ms_per_step'], d['roofline']['avg_launch_us'])"
  done
done
