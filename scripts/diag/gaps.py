"""Per-step kernel timeline from a rocprofv3 kernel trace (run_kernel_trace.csv): each kernel's start/end relative to
the step's first kernel, its queue, and the idle gap before it on its own queue and after the kernel it depends on.
Usage: python scripts/diag/gaps.py TRACE.csv [first-kernel-substring] [steps]"""
import csv
import statistics as st
import sys

KEYS = ("fwd_head", "conv_fwd", "conv_bwd_fc", "conv_bwd", "head16", "head_kernel", "l1_split", "wgrad_lds", "wgrad_sgd",
        "wgrad", "reduce_sgd_direct", "reduce_sgd", "reduce_direct", "reduce_slabs", "sgd_pack", "oneshot", "Fill", "copy")


def short(name):
    for k in KEYS:
        if k in name:
            return k
    return name[:24]


rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else None
nlast = int(sys.argv[3]) if len(sys.argv) > 3 else 3
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows)
ks = [k for k in ks if k[2] not in ("Fill", "copy")]
if first is None:  # the most frequent kernel that is first after the largest idle gap
    first = ks[0][2]
    for k in ("fwd_head", "conv_fwd", "l1_split", "head_kernel"):
        if any(x[2] == k for x in ks):
            first = k
            break
starts = [i for i, k in enumerate(ks) if k[2] == first]
periods, gaps = [], {}
for a, b in zip(starts, starts[1:]):
    stp = ks[a:b]
    t0 = stp[0][0]
    periods.append((ks[b][0] - t0) / 1e3)
    prev_end = {}
    for s, e, n, q in stp:
        g = (s - prev_end[q]) / 1e3 if q in prev_end else None
        if g is not None:
            gaps.setdefault(n, []).append(g)
        prev_end[q] = e
    last_end = max(e for _, e, _, _ in stp)
    gaps.setdefault("(step end -> next " + first + ")", []).append((ks[b][0] - last_end) / 1e3)
for a, b in list(zip(starts, starts[1:]))[-nlast:]:
    stp = ks[a:b]
    t0 = stp[0][0]
    print(f"step period {(ks[b][0] - t0) / 1e3:.2f} us")
    for s, e, n, q in stp:
        print(f"   q{q:>2} {n:18s} {(s - t0) / 1e3:8.2f} -> {(e - t0) / 1e3:8.2f}  ({(e - s) / 1e3:6.2f})")
print(f"median period over {len(periods)} steps: {st.median(periods):.2f} us")
for n, v in gaps.items():
    print(f"  median idle gap before {n:30s} on its queue: {st.median(v):6.2f} us")
