"""LDS bank model of conv_fwd_kernel<bf16> (csrc/kernels/lenet.hip): cycles per image per access kind.

Same bank rules as scripts/lds_model.py (cycles()).  Lane mappings are those of the kernel:
stage (ds_write_b128, 4 per thread), conv1 A fragments (ds_read_b128), conv1 epilogue stores
(p1s / p1c: 16-bit, m1s: 8-bit), conv2 A fragments (ds_read_b128), conv2 epilogue (p2s 16-bit, m2s 8-bit).
Overrides: python scripts/lds_model_fwd.py XP=1048 P1CP=232 M1CP=240
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from lds_model import BYTES, cycles  # noqa: E402


C1Q = (0, 1, 2, 3)  # conv1 M-row block -> pooled column (lenet.hip conv_fwd_kernel: identity)


def rup(x, m):
    return (x + m - 1) // m * m


def model(P):
    XP, P1CP, M1CP, RP = P["XP"], P["P1CP"], P["M1CP"], P.get("RP", 14)
    T = 2
    OFF_P1 = rup((8 * XP + 64) * T, 16)
    OFF_P1C = rup(OFF_P1 + 14 * RP * 8 * T, 16)
    OFF_M1 = rup(OFF_P1C + 6 * P1CP * T, 16)
    OFF_P2 = rup(OFF_M1 + 6 * M1CP, 16)
    OFF_M2 = rup(OFF_P2 + 400 * T, 16)
    acc = collections.defaultdict(lambda: [0, 0, 0, 0])

    def add(name, kind, addrs):
        c, ideal = cycles(kind, addrs)
        a = acc[name]
        a[0] += 1
        a[1] += c
        a[2] += ideal
        a[3] += len(addrs) * BYTES[kind]

    # stage: 4 waves, tid < 224, 4 x ds_write_b128
    for w in range(4):
        for q in range(4):
            addrs = {}
            for lane in range(64):
                tid = w * 64 + lane
                if tid >= 224:
                    continue
                sy, sg, sh = 2 + (tid >> 3), (tid >> 1) & 3, tid & 1
                addrs[lane] = ((4 * sh + q) * XP + sy * 32 + 8 * sg) * T
            add("stage xs (w128)", "w128", addrs)
    # conv1: per wave, 7 tiles: A reads (2 for tile 0, then 1 per tile), epilogue stores
    for w in range(4):
        for t in range(7):
            kcs = [0, 1] if t == 0 else [1]
            for kc in kcs:
                addrs = {}
                for lane in range(64):
                    row, grp = lane & 15, lane >> 4
                    q, e = C1Q[row >> 2], row & 3
                    xt = 2 * q + (e & 1)
                    addrs[lane] = (xt * XP + ((e >> 1) + 4 * kc + grp) * 32 + 8 * w + 128 * t) * T
                add("conv1 A (r128)", "r128", addrs)
            a1, a2, a3 = {}, {}, {}
            for lane in range(64):
                row, grp = lane & 15, lane >> 4
                n, r = row & 7, row >> 3
                if 4 * w + C1Q[grp] >= 14:
                    continue
                pp = (2 * t + r) * RP + 4 * w + C1Q[grp]
                a1[lane] = OFF_P1 + (pp * 8 + n) * T
                if n < 6:
                    yx = (2 * t + r) * 16 + 4 * w + C1Q[grp]
                    a2[lane] = OFF_P1C + (n * P1CP + yx) * T
                    a3[lane] = OFF_M1 + n * M1CP + yx
            add("conv1 epi p1s (w16)", "w16", a1)
            add("conv1 epi p1c (w16)", "w16", a2)
            add("conv1 epi m1s (w8)", "w8", a3)
    # conv2: waves 0-2 tiles (2w, 2w+1), wave 3 tile 6; 7 chunks each
    for w in range(4):
        mts = [2 * w, 2 * w + 1] if w < 3 else [6]
        for mt in mts:
            for kc in range(7):
                addrs = {}
                for lane in range(64):
                    row, grp = lane & 15, lane >> 4
                    q, e = row >> 2, row & 3
                    p = min(mt * 4 + q, 24)
                    py, px = p // 5, p % 5
                    base = ((2 * py + (e >> 1)) * RP + 2 * px + (e & 1)) * 8
                    pos = min(kc * 4 + grp, 24)
                    kh, kw = pos // 5, pos % 5
                    addrs[lane] = OFF_P1 + (base + (kh * RP + kw) * 8) * T
                add("conv2 A (r128)", "r128", addrs)
            a1, a2 = {}, {}
            for lane in range(64):
                row, grp = lane & 15, lane >> 4
                pp = mt * 4 + grp
                if pp < 25:
                    a1[lane] = OFF_P2 + (row * 25 + pp) * T
                    a2[lane] = OFF_M2 + row * 25 + pp
            add("conv2 epi p2s (w16)", "w16", a1)
            add("conv2 epi m2s (w8)", "w8", a2)
    # copy-outs: contiguous 16-byte reads (p1c, m1s, p2s, m2s), thread e reads chunk e
    for name, off, nbytes in (("copy p1c (r128)", OFF_P1C, 6 * P1CP * T), ("copy m1s (r128)", OFF_M1, 6 * M1CP),
                              ("copy p2s (r128)", OFF_P2, 400 * T), ("copy m2s (r128)", OFF_M2, 400)):
        n = nbytes // 16
        for w0 in range(0, n, 64):
            add(name, "r128", {lane: off + (w0 + lane) * 16 for lane in range(64) if w0 + lane < n})
    return acc


def report(P):
    acc = model(P)
    tot_c = tot_i = tot_b = 0
    print(f"{'access':24s} {'instr':>6s} {'cycles':>7s} {'ideal':>6s} {'conflict':>8s} {'bytes':>7s}")
    for name, (n, c, i, b) in acc.items():
        tot_c += c
        tot_i += i
        tot_b += b
        print(f"{name:24s} {n:6d} {c:7d} {i:6d} {100 * (c - i) / max(c, 1):7.1f}% {b:7d}")
    print(f"{'total':24s} {'':6s} {tot_c:7d} {tot_i:6d} {100 * (tot_c - tot_i) / max(tot_c, 1):7.1f}% {tot_b:7d}")


def search():
    """Pitch sweep: modelled total cycles per image (lower is better)."""
    res = []
    for XP in range(1024, 1120, 8):
        for RP in range(14, 22):
            for P1CP in (232, 240, 248, 256):
                for M1CP in (240, 256, 272, 288):
                    acc = model({"XP": XP, "P1CP": P1CP, "M1CP": M1CP, "RP": RP})
                    res.append((sum(v[1] for v in acc.values()), XP, RP, P1CP, M1CP))
    res.sort()
    for r in res[:8]:
        print("cycles %d  XP=%d RP=%d P1CP=%d M1CP=%d" % r)


if __name__ == "__main__":
    if sys.argv[1:] == ["search"]:
        search()
        sys.exit(0)
    P = {"XP": 1048, "P1CP": 232, "M1CP": 240}
    for arg in sys.argv[1:]:
        k, v = arg.split("=")
        P[k] = int(v)
    report(P)
