set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
L=gpurun_out/r1ao
mkdir -p $L
n=0
run() {  # label model batch env...
  n=$((n+1)); lab=$1; m=$2; b=$3; shift 3
  env "$@" timeout -k 10 200 python bench.py --model $m --batch $b --steps 2 --warmup 1 > $L/b_${lab}_$n.log 2>&1 || { echo "bench rc=$?"; tail -20 $L/b_${lab}_$n.log; exit 1; }
  echo "bench $lab $(tail -1 $L/b_${lab}_$n.log | python -c 'import sys,json; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
}
run xl512_ov gpt2-xl 512 DLMS_OVERLAP=1
run xl512_noov gpt2-xl 512 DLMS_OVERLAP=0
run xl512_cap8 gpt2-xl 512 DLMS_OVERLAP_SPLIT_CAP=8
run xl512_4p gpt2-xl 512 DLMS_OVERLAP_PARTS=4
run xl1024_ov gpt2-xl 1024 DLMS_OVERLAP=1
run med1024_noov gpt2-medium 1024 DLMS_OVERLAP=0
run med1024_cap8 gpt2-medium 1024 DLMS_OVERLAP_SPLIT_CAP=8
run med2048_ov gpt2-medium 2048 DLMS_OVERLAP=1
echo ALLDONE
