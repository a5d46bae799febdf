set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -m pytest tests/ -q -m gpu -p no:cacheprovider -rf -s > gpurun_out/tests.log 2>&1
echo "EXIT=$?" >> gpurun_out/tests.log
