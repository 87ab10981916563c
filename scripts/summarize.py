"""Summaries of gpurun_out artefacts: bench JSON lines, kernel stats, PMC counters."""
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


if __name__ == "__main__":
    kind, path = sys.argv[1], sys.argv[2]
    {"bench": bench, "stats": stats, "pmc": pmc}[kind](path)
