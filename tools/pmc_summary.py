"""Summarise tools/pmc_session.sh output into profiles/traffic_c2_b<B>.json.

Per-dispatch counter values are averaged per kernel; HBM bytes per k_decode launch (all
decode kernels of one bnflac_decode_parsed call) = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts
half the bytes of 16-B/lane reads, MI355X_MICROARCH.md) + WRITE_SIZE, both in KiB.
usage: python tools/pmc_summary.py gpurun_out/pmc_r1s B TAG > profiles/traffic_c2_b<B>.json
"""
import collections
import csv
import glob
import json
import os
import sys

d, B, tag = sys.argv[1], int(sys.argv[2]), sys.argv[3]
vals = collections.defaultdict(lambda: collections.defaultdict(list))
for f in sorted(glob.glob(os.path.join(d, "p*", "run_counter_collection.csv"))):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        short = name.split("(")[0].replace("void ", "")
        vals[short][r["Counter_Name"]].append(float(r["Counter_Value"]))
per = {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in vals.items()
       if k.startswith("k_decode") or k.startswith("k_parse")}
dec = [k for k in per if k.startswith("k_decode")]
fetch = sum(per[k].get("FETCH_SIZE", 0.0) for k in dec)
write = sum(per[k].get("WRITE_SIZE", 0.0) for k in dec)
out = {
    "workload": "C2", "batches_per_step": B, "frames_per_batch": 1024,
    "kernel": "k_decode launch = " + " + ".join(sorted(dec)),
    "fetch_size_kb_raw": fetch, "write_size_kb": write,
    "hbm_read_bytes": fetch * 1024 * 2, "hbm_write_bytes": write * 1024,
    "traffic_bytes": fetch * 1024 * 2 + write * 1024,
    "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half the bytes of 16-B/lane reads); "
                  "WRITE_SIZE as reported",
    "counters_per_kernel": per,
    "command": "tools/pmc_session.sh: rocprofv3 --pmc <one group per pass> -- python3 bench.py --steps 2 --warmup 1 "
               "--no-cpu-baseline --no-pcie --no-index",
    "round": tag,
}
print(json.dumps(out, indent=1))
