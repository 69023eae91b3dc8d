"""Per-kernel PMC table from tools/pmc_session.sh passes (any counters): average per dispatch,
plus per-wave figures when SQ_WAVES was collected.
usage: python tools/pmc_kernel.py gpurun_out/pmc_<tag> [kernel-prefix ...]"""
import collections
import csv
import glob
import os
import sys

d = sys.argv[1]
prefixes = sys.argv[2:] or ["k_"]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        short = r["Kernel_Name"].split("(")[0].replace("void ", "")
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k in sorted(vals):
    if not any(k.startswith(p) for p in prefixes):
        continue
    cs = {c: sum(v) / len(v) for c, v in vals[k].items()}
    waves = cs.get("SQ_WAVES")
    print(k)
    for c in sorted(cs):
        per = f"   per wave {cs[c] / waves:14.1f}" if waves and c != "SQ_WAVES" else ""
        print(f"  {c:28s} {cs[c]:18.1f}{per}")
