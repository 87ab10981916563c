"""Summaries of gpurun_out artefacts: bench JSON lines, kernel stats, PMC counters, kernel-trace timelines.

  python scripts/summarize.py gaps DIR/run_kernel_trace.csv [STEPS]   per-kernel start / end and the idle gap before
      each kernel (chip-wide: time since the latest end of any earlier kernel) over the last STEPS steps (default 3)
"""
import collections
import csv
import json
import sys


def bench(path):
    for l in open(path):
        l = l.strip()
        if not l.startswith("{"):
            continue
        d = json.loads(l)
        tune = d["config"].get("plan_autotune") or {}
        tm = " ".join(f"{k}={v}" for k, v in (tune.get("timings_ms") or {}).items())
        print(f"  {d['config']['model']:20s} {d['dtype']:5s} B={d['config']['per_gpu_batch']:6d} "
              f"{d['ms_per_step']:8.4f} ms/step {d['value']/1e6:8.3f} M img/s top1={d.get('top1')}"
              + (f" chosen={tune.get('chosen')} [{tm}]" if tune else ""))


def stats(path, n=10):
    rows = list(csv.DictReader(open(path)))
    for r in rows[:n]:
        print(f"  {int(r['Calls']):4d} {float(r['AverageNs'])/1000:9.2f}us {float(r['Percentage']):6.2f}%  {r['Name'][:70]}")


def pmc(path, pat=("conv", "head", "wgrad")):
    rows = list(csv.DictReader(open(path)))
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.defaultdict(set)
    for r in rows:
        k = r["Kernel_Name"][:48]
        agg[k][r["Counter_Name"]] += float(r["Counter_Value"])
        cnt[k].add(r["Dispatch_Id"])
    for k, v in agg.items():
        if any(p in k for p in pat):
            n = len(cnt[k])
            print("  " + k, " ".join(f"{c}={x / n:.3e}" for c, x in sorted(v.items())))


def _short(name):
    for k in ("conv_bwd_fc", "conv_bwd", "fwd_head", "conv_fwd", "head16", "head_kernel", "l1_split", "wgrad_sk",
              "wgrad_lds", "wgrad_sgd", "wgrad", "reduce_sgd_direct", "reduce_sgd", "reduce_direct", "reduce_slabs",
              "sgd_pack", "gather_next", "oneshot", "ncclDevKernel", "Fill", "copyBuffer"):
        if k in name:
            return k
    return name[:24]


def gaps(path, steps=3):
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), _short(r["Kernel_Name"]), r["Queue_Id"])
                 for r in rows))
    ks = [k for k in ks if k[2] not in ("Fill", "copyBuffer")]
    # a step starts at its first forward kernel
    firsts = [i for i, k in enumerate(ks) if k[2] in ("fwd_head", "conv_fwd", "head_kernel", "head16", "l1_split")
              and (i == 0 or ks[i - 1][2] not in ("conv_fwd", "l1_split"))]
    if len(firsts) < steps + 1:
        steps = max(1, len(firsts) - 1)
    sel = ks[firsts[-steps - 1]:firsts[-1]]
    t0, last_end = sel[0][0], sel[0][0]
    for s, e, n, q in sel:
        gap = (s - last_end) / 1000
        print(f"  q{q:>2s} {n:18s} start {(s - t0) / 1000:8.2f} end {(e - t0) / 1000:8.2f} dur {(e - s) / 1000:7.2f}"
              f"  gap {gap:6.2f} us")
        last_end = max(last_end, e)
    print(f"  {steps} steps: {(sel[-1][1] - t0) / 1000 / steps:.2f} us per step (last end)")


if __name__ == "__main__":
    if sys.argv[1] == "gaps":
        gaps(sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 3)
        sys.exit(0)
    kind, path = sys.argv[1], sys.argv[2]
    {"bench": bench, "stats": stats, "pmc": pmc}[kind](path)
