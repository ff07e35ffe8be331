# Wide-EP GPU check over several random checkpoints: flat (scale 1) vs sharpened
# (scale 8) routers. 2 processes share cuda:0 (scripts/ep_gpu_check.py).
set -o pipefail
mkdir -p gpurun_out/epdiag
export LLMD_SYMM_DEVICE=0 HSA_ENABLE_IPC_MODE_LEGACY=0
run() { # name port args...
  local name=$1 port=$2; shift 2
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=$port \
    scripts/ep_gpu_check.py --weights /tmp/epw_$name.safetensors "$@" > gpurun_out/epdiag/$name.log 2>&1
  local rc=$?
  echo "$name rc=$rc $(grep '^{' gpurun_out/epdiag/$name.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ok'], [[(x['pos'], x['margin'], x['near_tie']) for x in r['diverge']] for r in d['ranks']])")"
  if [ $rc -eq 124 ] || [ $rc -eq 137 ] || [ $rc -eq 134 ] || [ $rc -eq 139 ]; then exit $rc; fi
  return 0
}
port=29770
for model in tiny-gpt-oss tiny-deepseek; do
  for scale in 1 8; do
    for seed in 1 2 3 4 5 6; do
      port=$((port+1))
      extra=""; [ $model = tiny-deepseek ] && extra="--dbo --eplb"
      run ${model}_s${scale}_seed${seed} $port --model $model --seed $seed --router-scale $scale $extra || exit 1
    done
  done
done
