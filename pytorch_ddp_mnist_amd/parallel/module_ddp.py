"""``DistributedDataParallel`` for arbitrary torch modules (bring-your-own-model path).

Reference: ``DistributedDataParallel(model, device_ids=[rank], output_device=rank)``
(ddp_tutorial_multi_gpu.py:72) and ``DistributedDataParallel(model)`` (mnist_cpu_mp.py:371,
mnist_pnetcdf_cpu_mp.py:439); ``model.module`` unwrap (ddp_tutorial_multi_gpu.py:118).  The two
fixed models of the reference run on the native engine (csrc/runtime/trainer.cpp), where the
kernels write gradients straight into the bucket slab.  This wrapper gives the same DDP contract
to any other ``nn.Module`` a user brings, so switching from ``torch.nn.parallel.DDP`` is a
one-line change:

  * parameters (and buffers) are broadcast from rank 0 at construction;
  * gradients live in ONE flat fp32 slab laid out in *reverse* registration order (the order
    backward produces them), and every ``param.grad`` is a view into it (torch's
    ``gradient_as_bucket_view=True``), so a bucket is a contiguous slice: no flatten/copy;
  * a post-accumulate-grad hook counts each bucket down; the moment its last gradient lands the
    bucket's SUM all-reduce is enqueued on a side stream (native :class:`RcclComm` over xGMI on
    MI355X, c10d otherwise) while backward keeps running on the compute stream;
  * an autograd end-of-backward callback launches buckets whose parameters got no gradient
    (zeros, like ``find_unused_parameters``), joins the side stream and scales by 1/world;
  * ``no_sync()`` skips communication for gradient accumulation, as torch's DDP does.

Bucket sizes: the first bucket is capped at 1 MiB and later ones at ``bucket_cap_mb`` (torch's
defaults, reducer.cpp), but the default cap here is 4 MiB rather than 25 MiB: on an 8-GPU xGMI
ring each ring step moves bucket/8 over one 153 GB/s link, so a 4 MiB bucket costs ~5 us per
step, small enough to hide behind backward while keeping per-collective launch latency rare.
"""
from __future__ import annotations

import contextlib
from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


class _Bucket:
    __slots__ = ("lo", "hi", "params", "pending", "launched", "work")

    def __init__(self, lo: int, hi: int, params: List[torch.nn.Parameter]):
        self.lo, self.hi, self.params = lo, hi, params
        self.pending = len(params)
        self.launched = False
        self.work = None


def assign_buckets(sizes: Sequence[int], elem_bytes: int = 4, first_cap: int = 1 << 20,
                   cap: int = 4 << 20) -> List[List[int]]:
    """Group parameter indices (given in backward order) into consecutive size-capped buckets.

    A parameter never straddles buckets; one larger than the cap gets its own bucket.
    """
    out: List[List[int]] = []
    cur: List[int] = []
    cur_bytes = 0
    limit = first_cap
    for i, n in enumerate(sizes):
        b = n * elem_bytes
        if cur and cur_bytes + b > limit:
            out.append(cur)
            cur, cur_bytes, limit = [], 0, cap
        cur.append(i)
        cur_bytes += b
    if cur:
        out.append(cur)
    return out


class DistributedDataParallel(torch.nn.Module):
    def __init__(self, module: torch.nn.Module, device_ids: Optional[Sequence[int]] = None,
                 output_device: Optional[int] = None, bucket_cap_mb: float = 4.0,
                 first_bucket_mb: float = 1.0, rccl=None, process_group=None,
                 broadcast_buffers: bool = True):
        super().__init__()
        self.module = module
        self.device_ids = list(device_ids) if device_ids else None
        self.output_device = output_device
        self.rccl = rccl
        self.pg = process_group
        self.world = rccl.world if rccl is not None else (
            dist.get_world_size(process_group) if dist.is_available() and dist.is_initialized() else 1)
        self.broadcast_buffers = broadcast_buffers
        self._sync = True
        self._params = [p for p in module.parameters() if p.requires_grad]
        if not self._params:
            raise ValueError("DistributedDataParallel: module has no parameters that require grad")
        dev = self._params[0].device
        if any(p.device != dev for p in self._params):
            raise ValueError("DistributedDataParallel: all parameters must be on one device")
        if any(p.dtype != torch.float32 for p in self._params):
            raise ValueError("DistributedDataParallel: fp32 master parameters expected")
        self.device = dev
        order = list(reversed(range(len(self._params))))  # backward order
        groups = assign_buckets([self._params[i].numel() for i in order], 4,
                                int(first_bucket_mb * (1 << 20)), int(bucket_cap_mb * (1 << 20)))
        total = sum(p.numel() for p in self._params)
        self.grad_slab = torch.zeros(total, dtype=torch.float32, device=dev)
        self._views = {}
        self.buckets: List[_Bucket] = []
        self._bucket_of = {}
        off = 0
        for g in groups:
            lo = off
            ps = []
            for j in g:
                p = self._params[order[j]]
                n = p.numel()
                self._views[p] = self.grad_slab[off:off + n].view_as(p)
                off += n
                ps.append(p)
            b = _Bucket(lo, off, ps)
            for p in ps:
                self._bucket_of[p] = b
            self.buckets.append(b)
        for p in self._params:
            p.grad = self._views[p]
        self._comm_stream = torch.cuda.Stream(device=dev) if dev.type == "cuda" else None
        self._callback_queued = False
        self._hooks = [p.register_post_accumulate_grad_hook(self._on_grad) for p in self._params]
        self._broadcast_state()

    # ------------------------------------------------------------------ construction
    def _broadcast_state(self) -> None:
        if self.world <= 1 and self.rccl is None:
            return
        with torch.no_grad():
            tensors = [p.data for p in self._params]
            if self.broadcast_buffers:
                tensors += [b for b in self.module.buffers()]
            for t in tensors:
                self._broadcast(t)

    def _broadcast(self, t: torch.Tensor) -> None:
        if self.rccl is not None and t.dtype == torch.float32 and t.is_contiguous():
            s = torch.cuda.current_stream(self.device)
            self.rccl.broadcast_f32(t.data_ptr(), t.numel(), 0, s.cuda_stream)
        else:
            dist.broadcast(t, 0, group=self.pg)

    # ------------------------------------------------------------------ forward
    def forward(self, *args, **kwargs):
        if torch.is_grad_enabled():
            for b in self.buckets:
                b.pending, b.launched, b.work = len(b.params), False, None
            self._callback_queued = False
        return self.module(*args, **kwargs)

    @contextlib.contextmanager
    def no_sync(self):
        """Accumulate local gradients without all-reducing (torch DDP's no_sync)."""
        old, self._sync = self._sync, False
        try:
            yield
        finally:
            self._sync = old

    # ------------------------------------------------------------------ backward hooks
    def _on_grad(self, p: torch.Tensor) -> None:
        view = self._views[p]
        if p.grad is not view:  # zero_grad(set_to_none=True) dropped the view: re-bind it
            view.copy_(p.grad)
            p.grad = view
        if not self._sync or (self.world <= 1 and self.rccl is None):
            return  # an explicitly attached RcclComm is used even at world 1 (as the native trainer does)
        if not self._callback_queued:
            self._callback_queued = True
            torch.autograd.Variable._execution_engine.queue_callback(self._finish)
        b = self._bucket_of[p]
        b.pending -= 1
        if b.pending == 0 and not b.launched:
            self._launch(b)

    def _launch(self, b: _Bucket) -> None:
        b.launched = True
        flat = self.grad_slab[b.lo:b.hi]
        if self._comm_stream is not None:
            # the bucket's last gradient was produced on the compute stream: order the side stream after it
            self._comm_stream.wait_stream(torch.cuda.current_stream(self.device))
            if self.rccl is not None:
                self.rccl.all_reduce_sum_f32(flat.data_ptr(), flat.numel(), self._comm_stream.cuda_stream)
            else:
                with torch.cuda.stream(self._comm_stream):
                    b.work = dist.all_reduce(flat, group=self.pg, async_op=True)
        else:
            b.work = dist.all_reduce(flat, group=self.pg, async_op=True)

    def _finish(self) -> None:
        for b in self.buckets:
            if not b.launched:  # parameters unused in this forward: contribute zeros
                for p in b.params:
                    if p.grad is None:
                        p.grad = self._views[p]
                        p.grad.zero_()
                self._launch(b)
        for b in self.buckets:
            if b.work is not None:
                b.work.wait()
                b.work = None
        if self._comm_stream is not None:
            torch.cuda.current_stream(self.device).wait_stream(self._comm_stream)
        self.grad_slab.div_(self.world)
        self._callback_queued = False

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []


DDP = DistributedDataParallel
