set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -q -m gpu -p no:cacheprovider -rf -k "${TK:-attention or rmsnorm or rope}" > gpurun_out/q_tests.log 2>&1 || { echo "TESTS FAILED"; tail -40 gpurun_out/q_tests.log; exit 1; }
tail -2 gpurun_out/q_tests.log
