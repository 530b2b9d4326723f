set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1o
mkdir -p $L
scripts/gpu_step.sh 560 $L/cfg2.log python scripts/run_config.py --config 2 --students 48 --queries 2 --workdir $L/cfg2 || exit 1
scripts/gpu_step.sh 300 $L/vendor.log python scripts/bench_kernels.py --batches=256,1024 --tiles=-1 --vendor --ops qkv,oproj,fc,proj,lmhead || exit 1
scripts/gpu_step.sh 300 $L/pmc1.log rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS -d $L/pmc1 -o run -- python3 scripts/bench_kernels.py --batches=256 --tiles=-1 --ops qkv,lmhead || exit 1
scripts/gpu_step.sh 300 $L/pmc2.log rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_LATENCY_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum TA_BUSY_avr -d $L/pmc2 -o run -- python3 scripts/bench_kernels.py --batches=256 --tiles=-1 --ops qkv,lmhead || exit 1
echo ALLDONE
