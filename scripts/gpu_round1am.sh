set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1am
mkdir -p $L
T=-1,0,1,2,3,4,5,6,7,9,10,11,12,13,14
timeout -k 10 400 python scripts/bench_kernels.py --d 1600 --batches=256,512 --tiles=$T --ops qkv,oproj,fc,proj > $L/xl.log 2>&1 || { echo "rc=$?"; tail -20 $L/xl.log; exit 1; }
echo XL; grep '^{' $L/xl.log | cut -c1-110
timeout -k 10 400 python scripts/bench_kernels.py --d 1024 --batches=512 --tiles=$T --ops qkv,oproj,fc,proj > $L/med.log 2>&1 || { echo "rc=$?"; tail -20 $L/med.log; exit 1; }
echo MED; grep '^{' $L/med.log | cut -c1-110
timeout -k 10 300 python bench.py --model gpt2-xl --batch 512 --steps 2 --warmup 1 > $L/bench_xl.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/bench_xl.log; exit 1; }
echo "bench xl $(tail -1 $L/bench_xl.log | cut -c90-190)"
echo ALLDONE
