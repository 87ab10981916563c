"""Register / scratch / occupancy summary of the HIP kernels (hipcc -Rpass-analysis=kernel-resource-usage).
Usage: python scripts/kres.py csrc/kernels/head.hip [name-filter]"""
import re
import subprocess
import sys

src = sys.argv[1]
filt = sys.argv[2] if len(sys.argv) > 2 else ""
r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-Icsrc", "-c", src, "-o",
                    "/tmp/_kres.o", "-Rpass-analysis=kernel-resource-usage"], capture_output=True, text=True)
cur, rows = None, []
for line in r.stderr.splitlines():
    m = re.search(r"remark: (.*?): (.*) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        cur = {"name": subprocess.run(["c++filt"], input=v, capture_output=True, text=True).stdout.strip()}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for d in rows:
    n = d["name"]
    if filt not in n:
        continue
    n = re.sub(r"\(anonymous namespace\)::", "", n)
    n = re.sub(r"HeadDims<784[^>]*>", "MLP", n)
    n = re.sub(r"HeadDims<400[^>]*>", "LeNet", n)
    n = n.split("(")[0]
    print(f"{n[:70]:70s} vgpr {d.get('VGPRs', '?'):>4} agpr {d.get('AGPRs', '?'):>3} scratch {d.get('ScratchSize [bytes/lane]', '?'):>4} "
          f"occ {d.get('Occupancy [waves/SIMD]', '?'):>2} lds {d.get('LDS Size [bytes/block]', '?')}")
