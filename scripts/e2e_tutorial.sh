set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29611 ddp_tutorial_multi_gpu.py --synthetic > gpurun_out/e2e_mlp.log 2>&1 &&
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29612 ddp_tutorial_multi_gpu.py --synthetic --model lenet5 --dtype bf16 > gpurun_out/e2e_lenet.log 2>&1
echo rc=$?
