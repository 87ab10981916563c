"""Summarise scripts/ablate.sh runs: mean time of the conv kernels per ablation mask."""
import csv
import glob
import os
import sys

tag = sys.argv[1]
rows = []
for d in glob.glob(f"{tag}_*"):
    if not os.path.isdir(d):
        continue
    m = int(d.rsplit("_", 1)[1])
    st = {}
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_stats.csv"))):
        for k in ("conv_bwd", "conv_fwd"):
            if k in r["Name"]:
                st[k] = float(r["AverageNs"]) / 1000
    rows.append((m, st))
for m, st in sorted(rows):
    print(f"mask {m:5d}  conv_fwd {st.get('conv_fwd', 0):7.2f} us  conv_bwd {st.get('conv_bwd', 0):7.2f} us")
