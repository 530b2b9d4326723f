set -e
cd /tmp && export TMPDIR=/tmp
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmc_lab
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES -d gpurun_out/pmc_lab -o pass2 --output-format csv -- ./scripts/gemm_lab qkv > gpurun_out/pmc_lab/lab.out 2>&1
echo done1
ls -R gpurun_out/pmc_lab | head
