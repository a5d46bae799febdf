set -o pipefail
mkdir -p gpurun_out/pmc2
export TMPDIR=/tmp
run() { # tag env...
  tag=$1; shift
  env "$@" timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC --output-format csv -d gpurun_out/pmc2/${tag}_A -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc2/err.log || echo "fail $tag A" >> gpurun_out/pmc2/err.log
  env "$@" timeout -k 10 120 rocprofv3 --pmc SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE --output-format csv -d gpurun_out/pmc2/${tag}_B -o p -- python tools/gemm_one.py > /dev/null 2>>gpurun_out/pmc2/err.log || echo "fail $tag B" >> gpurun_out/pmc2/err.log
}
run v0q GO_VARIANT=0
run v1q GO_VARIANT=1
run blas GO_VARIANT=0 GO_BLAS=1
run v0o GO_VARIANT=0 GO_SHAPE=4800,4096,4096,64
echo done
