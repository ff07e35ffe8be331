set -o pipefail
mkdir -p gpurun_out
export LLMD_SYMM_DEVICE=0
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 \
    --master-port=$((29700 + RANDOM % 200)) scripts/ep_gpu_check.py "$@" > gpurun_out/ep_$name.log 2>&1 \
    || { echo "ep check $name failed"; tail -40 gpurun_out/ep_$name.log; return 1; }
  grep '^{' gpurun_out/ep_$name.log
}
run base && run dbo --dbo && run dbo_eager --dbo --dbo-eager && run eplb --eplb && run deepseek_dbo --model tiny-deepseek --dbo && run deepseek_eplb_dbo --model tiny-deepseek --dbo --eplb
