# fused decode Linear: generate tests, T2I bench (fused default vs round-2 step), kernel stats
set -o pipefail
timeout -k 10 600 python -u -m pytest tests/test_gpu_generate.py -q -x -p no:cacheprovider --timeout 300 --timeout-method thread -s > gpurun_out/dl_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/dl_tests.log; exit 1; }
tail -1 gpurun_out/dl_tests.log
grep -E "folded|fused vs|T2I" gpurun_out/dl_tests.log | head
timeout -k 10 400 python -u bench.py --workload t2i --no-cpu-baseline > gpurun_out/dl_t2i.json 2> gpurun_out/dl_t2i.err || { echo "T2I BENCH FAILED"; tail -5 gpurun_out/dl_t2i.err; exit 1; }
cut -c1-600 gpurun_out/dl_t2i.json
timeout -k 10 400 python -u bench.py --workload t2i --no-cpu-baseline --t2i-unfused > gpurun_out/dl_t2i_old.json 2> gpurun_out/dl_t2i_old.err || { echo "T2I BENCH FAILED"; tail -5 gpurun_out/dl_t2i_old.err; exit 1; }
cut -c1-600 gpurun_out/dl_t2i_old.json
