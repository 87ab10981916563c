"""Per-phase wall-clock stamps of the fused head kernel (MNIST_AMD_STAMPS=1).

Runs the headline config (LeNet-5 bf16, B=8192) for a few steps, then prints, over the head
workgroups of the last step, the mean/min/max duration of each phase (stamp k -> k+1) and the
spread of workgroup start/end times.  The wall clock ticks at 100 MHz (10 ns).
"""
import os
import sys

os.environ["MNIST_AMD_STAMPS"] = "1"
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import numpy as np  # noqa: E402
import torch  # noqa: E402

from pytorch_ddp_mnist_amd.data.synthetic import make_split  # noqa: E402
from pytorch_ddp_mnist_amd.engine.native import NativeTrainer  # noqa: E402
from pytorch_ddp_mnist_amd.models import build_model  # noqa: E402

B = int(os.environ.get("STAMP_BATCH", "8192"))
model = os.environ.get("STAMP_MODEL", "lenet5")
dtype = os.environ.get("STAMP_DTYPE", "bf16")
x, y = make_split(60000, seed=1)
dev = torch.device("cuda", 0)
tr = NativeTrainer(model, dtype, B, torch.from_numpy(x.reshape(-1, 784)).to(dev), torch.from_numpy(y).to(dev),
                   device=dev, lr=0.05, momentum=0.9, dropout=0.0, init=build_model(model))
tr.set_epoch_indices(torch.randperm(60000, dtype=torch.int32)[: (60000 // B) * B])
tr.reset_metrics()
for _ in range(6):
    tr.step(B, use_graph=True)
tr.synchronize()
allst = tr.stamps.view(-1, 16).cpu().numpy().astype(np.int64)


def report(title, st, names, last):
    """st: [blocks][16] stamps; names[k] = phase between stamp k and k+1; `last` = final stamp slot."""
    t0 = st[:, 0].min()
    print(f"{title}: {len(st)} workgroups; start spread {(st[:, 0].max() - t0) * 10 / 1000:.2f} us; "
          f"span {(st[:, last].max() - t0) * 10 / 1000:.2f} us")
    for k, n in enumerate(names):
        if n is None:
            continue
        d = (st[:, k + 1] - st[:, k]) * 10 / 1000.0
        print(f"  {n:16s} mean {d.mean():7.2f} us  min {d.min():7.2f}  max {d.max():7.2f}")
    tot = (st[:, last] - st[:, 0]) * 10 / 1000.0
    print(f"  {'total':16s} mean {tot.mean():7.2f} us  min {tot.min():7.2f}  max {tot.max():7.2f}")


def per_cu(title, st, loc, last):
    """Balance across compute units: each CU's finish time (its last workgroup's final stamp)
    relative to the kernel's first start.  loc = XCC << 32 | HW_ID per workgroup."""
    hw = loc & 0xFFFFFFFF
    key = ((loc >> 32) & 15) * 4096 + ((hw >> 13) & 7) * 512 + ((hw >> 12) & 1) * 256 + ((hw >> 8) & 15)
    t0 = st[:, 0].min()
    end = (st[:, last] - t0) * 10 / 1000.0
    cus = {}
    for k, e in zip(key.tolist(), end.tolist()):
        n, m = cus.get(k, (0, 0.0))
        cus[k] = (n + 1, max(m, e))
    fin = np.array([m for _, m in cus.values()])
    nwg = np.array([n for n, _ in cus.values()])
    xccs = sorted({k // 4096 for k in cus})
    per_xcc = " ".join(f"x{x}:{max(m for k, (_, m) in cus.items() if k // 4096 == x):.1f}" for x in xccs)
    rr = np.mean(((loc >> 32) & 15) == (np.arange(len(loc)) % 8))
    print(f"{title}: workgroup g on XCD g % 8 for {100 * rr:.1f}% of workgroups")
    print(f"{title} per-CU: {len(cus)} CUs, workgroups/CU min {nwg.min()} max {nwg.max()}; CU finish "
          f"mean {fin.mean():.2f} us  min {fin.min():.2f}  p90 {np.percentile(fin, 90):.2f}  max {fin.max():.2f}; "
          f"per-XCC max {per_xcc}")


# head rows per workgroup (head.hip head_rows_per_block; the split path at small batches uses 16)
if B <= tr.C.L1_SPLIT_MAX_B and model == "mlp" or B <= 256:
    rows = 16
else:
    rows = 32
nblk = (B + rows - 1) // rows
fused = tr.fwd_head_applies() and tr.rt.fwd_head
if fused:  # fwd_head_kernel: 16-row workgroups; head rows hold the head phases after the conv loops
    nblk = B // 16
    st = allst[:nblk][:, [0, 9, 1, 2, 3, 4, 5, 6, 7, 8]]
    report("fwd_head (head part)", st, ["X^T + L1 issue", "L1", "L2", "L3", "softmax", "dH2", "dH1", "dX", "dX store"], 9)
    report("fwd_head (conv loops, half 0)", allst[2048:2048 + min(nblk, 1024)],
           ["setup"] + [f"img{t} {p}" for t in range(4) for p in ("stage", "conv1", "conv2")], 14)
    fw = allst[2048:2048 + nblk]
    print(f"  conv loop start -> head end: {((allst[:nblk, 8] - fw[:, 0]) * 10 / 1000).mean():.2f} us mean")
    whole = np.concatenate([fw[:, :1], allst[:nblk, 8:9]], axis=1)  # [conv loop start, head end]
    per_cu("fwd_head", whole, fw[:, 15], 1)
    nb = 512
    bw = allst[1024:1024 + nb]
    print(f"boundaries: fwd_head last end -> conv_bwd first start {(bw[:, 0].min() - allst[:nblk, 8].max()) * 10 / 1000:.2f} us; "
          f"fwd_head first start -> conv_bwd last end {(bw[:, 15].max() - fw[:, 0].min()) * 10 / 1000:.2f} us")
    bnames = ["setup"]
    for t in range(4):
        bnames += [f"img{t} A (stage)", f"img{t} B (w2+dgrad)", f"img{t} C (w1)"]
    report("conv_bwd", bw, bnames + [None, "slab write"], 15)
    per_cu("conv_bwd", bw, allst[4608:4608 + nb, 0], 15)
    wg = allst[3072:3584]
    wg = wg[wg[:, 0] > 0]
    if len(wg) and (wg[:, 3] > 0).all():  # wgrad_sk: [1] K loop done, [2] reduced + stored, [3] location + 1
        report("wgrad", wg, ["loads + MFMA", "reduce + store"], 2)
        per_cu("wgrad", wg, wg[:, 3] - 1, 2)
        print(f"  fwd_head last end -> wgrad first start {(wg[:, 0].min() - allst[:nblk, 8].max()) * 10 / 1000:.2f} us; "
              f"wgrad last end -> conv_bwd first start {(bw[:, 0].min() - wg[:, 2].max()) * 10 / 1000:.2f} us")
elif model == "lenet5":
    report("head", allst[:nblk], ["idx+stage X", "L1", "L2", "L3", "softmax", "dH2", "dH1", "dX"], 8)
    # inside the staging phase: [0] entry -> [9] loads issued -> [10] weights stored -> [11] X stored -> [1] barrier
    hs = allst[:nblk][:, [0, 9, 10, 11, 1]]
    if (hs[:, 1:4] > 0).all():
        report("head staging", hs, ["issue loads", "wait+W stores", "X stores", "barrier"], 4)
    # inside the softmax phase: [4] start -> [12] dX loads issued -> [13] rows done -> [14] partials -> [5] barrier
    ss = allst[:nblk][:, [4, 12, 13, 14, 5]]
    if (ss[:, 1:4] > 0).all():
        report("head softmax", ss, ["dX prefetch", "softmax rows", "metric sums", "barrier"], 4)
        pw = allst[4096:4096 + nblk, :16]  # STAMP_HEAD_ARRIVE
        if (pw > 0).all():
            rel = (pw - allst[:nblk, 4][:, None]) * 10 / 1000.0
            print("  per-wave arrival at the softmax barrier (us after phase start): " +
                  " ".join(f"w{i}:{rel[:, i].mean():.2f}" for i in range(16)))
else:  # no dX phase: stamp 7 is never written, dH1 ends at stamp 8
    allst[:nblk, 7] = allst[:nblk, 8]
    report("head", allst[:nblk], ["idx+stage X", "L1", "L2", "L3", "softmax", "dH2", "dH1"], 8)
    # MLP staging: [0] entry -> [9] idx + bias loads issued -> [10] (no LDS weights) -> barrier + gather +
    # convert + stores -> [11] -> [1] barrier
    hs = allst[:nblk][:, [0, 9, 11, 1]]
    if (hs[:, 1:3] > 0).all():
        report("head staging", hs, ["idx/bias issue", "gather+convert+X/xT stores", "barrier"], 3)
if model == "lenet5" and not fused:
    per_img = []
    for t in range(4):
        per_img += [f"img{t} stage" if t == 0 else f"img{t} stage(+prev)", f"img{t} conv1", f"img{t} conv2"]
    nf = (B + 7) // 8 if B >= 1024 else B
    report("conv_fwd", allst[2048:2048 + min(nf, 1024)], ["setup"] + per_img, 14)
    nb = 512 if B >= 512 else B
    bnames = ["setup"]
    for t in range(4):
        bnames += [f"img{t} A (stage)", f"img{t} B (w2+dgrad)", f"img{t} C (w1)"]
    report("conv_bwd", allst[1024:1024 + nb], bnames + [None, "slab write"], 15)

    # kernel boundaries on the device clock: last workgroup end of one kernel -> first start of the next
    fw, hd, bw = allst[2048:2048 + min(nf, 1024)], allst[:nblk], allst[1024:1024 + nb]
    print(f"boundaries: conv_fwd last end -> head first start {(hd[:, 0].min() - fw[:, 14].max()) * 10 / 1000:.2f} us; "
          f"head last end -> conv_bwd first start {(bw[:, 0].min() - hd[:, 8].max()) * 10 / 1000:.2f} us; "
          f"conv_fwd first start -> conv_bwd last end {(bw[:, 15].max() - fw[:, 0].min()) * 10 / 1000:.2f} us")
    per_cu("conv_fwd", allst[2048:2048 + min(nf, 1024)], allst[2048:2048 + min(nf, 1024), 15], 14)
    per_cu("conv_bwd", allst[1024:1024 + nb], allst[4608:4608 + nb, 0], 15)  # hw location: STAMP_BWD_HWLOC
    per_cu("head", allst[:nblk], allst[:nblk, 15], 8)
    wg = allst[3072:3584]
    wg = wg[wg[:, 0] > 0]
    if len(wg):  # FC weight gradient (aux stream beside conv_bwd, or between head and conv_bwd when serial)
        print(f"wgrad: {len(wg)} workgroups; head last end -> wgrad first start {(wg[:, 0].min() - hd[:, 8].max()) * 10 / 1000:.2f} us; "
              f"wgrad span {(wg[:, 1].max() - wg[:, 0].min()) * 10 / 1000:.2f} us; wgrad last end -> conv_bwd first start "
              f"{(bw[:, 0].min() - wg[:, 1].max()) * 10 / 1000:.2f} us")

if model == "mlp":
    def live(st):
        return st[st[:, 0] > 0]
    l1s, hs, wgs = live(allst[3584:4096]), allst[:nblk], live(allst[3072:3584])
    wlast = 2 if (wgs[:, 2] > 0).all() else 1   # wgrad_sgd / wgrad_sk stamps 0..2, the split wgrad 0..1
    sk = (wgs[:, 3] > 0).all()                  # wgrad_sk: [1] K loop done, [2] block reduced + stored, [3] location
    report("wgrad", wgs, (["loads + MFMA", "reduce + store"] if sk else ["GEMM", "epilogue"])[:wlast], wlast)
    if sk:
        per_cu("wgrad per CU", wgs, wgs[:, 3] - 1, 2)
    if len(l1s):
        report("l1_split", l1s, ["stage X", "GEMM"], 2)
    T0 = (l1s if len(l1s) else hs)[:, 0].min()
    for name, st, last in (("l1_split", l1s, 2), ("head", hs, 8), ("wgrad", wgs, wlast)):
        if not len(st):
            continue
        print(f"{name:9s} first start {(st[:, 0].min() - T0) * 10 / 1000:6.2f} us  last start "
              f"{(st[:, 0].max() - T0) * 10 / 1000:6.2f}  last end {(st[:, last].max() - T0) * 10 / 1000:6.2f}")
