# P/D same-device check (tiny-gpt-oss, hybrid KV), printed in full
set -o pipefail
mkdir -p gpurun_out
LLMD_PD_DEVICES=0,0 LLMD_KV_VMM=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29611 scripts/pd_check.py --model tiny-gpt-oss --transport ipc > gpurun_out/r5q_pd.out 2> gpurun_out/r5q_pd.err
rc=$?; grep PDCHECK gpurun_out/r5q_pd.out; grep -v "Gloo\|amdgpu.ids\|socket.cpp" gpurun_out/r5q_pd.err | grep -i "error\|Traceback" | head -10
LLMD_ATTN_OVERLAP=0 LLMD_PD_DEVICES=0,0 LLMD_KV_VMM=1 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr=127.0.0.1 --master-port=29612 scripts/pd_check.py --model tiny-gpt-oss --transport ipc > gpurun_out/r5q_pd0.out 2> gpurun_out/r5q_pd0.err
rc2=$?; echo "no overlap:"; grep PDCHECK gpurun_out/r5q_pd0.out
exit 0
