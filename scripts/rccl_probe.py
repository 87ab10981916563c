"""Diagnose RCCL bring-up on a box: torch's own nccl PG (world 1) vs the native RcclComm."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

which = sys.argv[1]
if which == "torch":
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT="29711")
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    x = torch.ones(10, device="cuda")
    dist.all_reduce(x)
    torch.cuda.synchronize()
    print("torch nccl ok", x.sum().item(), torch.cuda.nccl.version())
    dist.destroy_process_group()
else:
    from pytorch_ddp_mnist_amd.ops.native import load_c
    C = load_c()
    print("rccl version", C.rccl_version(), flush=True)
    uid = C.RcclComm.make_unique_id()
    print("uid ok", len(uid), flush=True)
    comm = C.RcclComm(uid, 0, 1, 0)
    print("comm ok", flush=True)
    x = torch.ones(10, device="cuda")
    comm.all_reduce_sum_f32(x.data_ptr(), 10, torch.cuda.current_stream().cuda_stream)
    torch.cuda.synchronize()
    print("native rccl ok", x.sum().item())
