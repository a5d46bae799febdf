set -o pipefail
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pvar -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline --lora-variant da_stream,swiglu_u > gpurun_out/pvar.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/pvar.log; exit 1; }
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/pbase -o p -- python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/pbase.log 2>&1 || { echo "PROF FAILED"; tail -5 gpurun_out/pbase.log; exit 1; }
echo prof ok
