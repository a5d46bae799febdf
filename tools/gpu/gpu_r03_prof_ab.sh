set -o pipefail
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_new -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pab_new.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/pab_new.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pab_r2 -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --round2-lora > gpurun_out/pab_r2.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/pab_r2.log; exit 1; }
echo prof ok
