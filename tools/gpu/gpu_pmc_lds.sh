set -o pipefail
mkdir -p gpurun_out/pmc_lds
export TMPDIR=/tmp
for V in 0; do
  GO_VARIANT=$V GO_ITERS=10 timeout -k 10 180 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAIT_INST_LDS --output-format csv -d gpurun_out/pmc_lds/v${V} -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc_lds/err.log || { echo "fail"; exit 1; }
  GO_VARIANT=$V GO_ITERS=10 timeout -k 10 180 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/pmc_lds/w${V} -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc_lds/err.log || { echo "fail"; exit 1; }
done
echo done
