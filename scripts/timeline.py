"""Per-step critical-path timeline from a rocprofv3 kernel trace (csv): for the last N steps, each
kernel's start/end relative to the step's conv_fwd start and the idle gaps on the main chain."""
import csv
import sys


def short(name):
    for k in ("conv_fwd", "conv_bwd", "head_kernel", "wgrad", "reduce_sgd_direct", "reduce_sgd", "reduce_direct",
              "reduce_kernel", "sgd_pack", "l1_split", "Fill", "copy"):
        if k in name:
            return k
    return name[:30]


rows = list(csv.DictReader(open(sys.argv[1])))
nlast = int(sys.argv[2]) if len(sys.argv) > 2 else 5
ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), short(r["Kernel_Name"]), r["Queue_Id"]) for r in rows))
starts = [i for i, k in enumerate(ks) if k[2] == "conv_fwd"]
steps = []
for a, b in zip(starts, starts[1:] + [len(ks)]):
    steps.append(ks[a:b])
tot = []
for st in steps[-nlast - 1:-1]:
    t0 = st[0][0]
    nxt = steps[steps.index(st) + 1][0][0]
    print(f"step period {(nxt - t0) / 1e3:.2f} us")
    for s, e, n, q in st:
        print(f"   q{q} {n:18s} {(s - t0) / 1e3:8.2f} -> {(e - t0) / 1e3:8.2f}  ({(e - s) / 1e3:6.2f})")
    tot.append((nxt - t0) / 1e3)
periods = [(steps[i + 1][0][0] - steps[i][0][0]) / 1e3 for i in range(len(steps) - 1)]
print("periods:", " ".join(f"{p:.1f}" for p in periods))
