"""Summarise tools/pmc_session.sh output into profiles/traffic_<cfg>_b<B>.json.

Per-dispatch counter values are averaged per kernel; HBM bytes per decode launch (all
decode kernels of one bnflac_decode_parsed call) = FETCH_SIZE x 2 (gfx950: FETCH_SIZE counts
half the bytes of 16-B/lane reads, MI355X_MICROARCH.md; tools/ubench_fetch.hip checks the
same factor for the decoders' per-lane LDS-DMA groups) + WRITE_SIZE, both in KiB.  The
kernel sources' hash ties the summary to the build bench.py times (bench.measured_traffic).
usage: python tools/pmc_summary.py gpurun_out/pmc_<tag> <cfg> <B> <frames> <tag> > profiles/traffic_<cfg>_b<B>.json
"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

d, cfg, B, frames, tag = sys.argv[1], sys.argv[2], int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
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
    "workload": cfg, "batches_per_step": B, "frames_per_batch": frames, "kernels_sha": bench.kernels_sha(),
    "kernel": "decode launch = " + " + ".join(sorted(dec)),
    "fetch_size_kb_raw": fetch, "write_size_kb": write,
    "hbm_read_bytes": fetch * 1024 * 2, "hbm_write_bytes": write * 1024,
    "traffic_bytes": fetch * 1024 * 2 + write * 1024,
    "correction": "FETCH_SIZE x2 (MI355X_MICROARCH.md: gfx950 FETCH_SIZE reports half the bytes of 16-B/lane reads; "
                  "profiles/ubench_fetch_*.txt for the per-lane LDS-DMA shape); WRITE_SIZE as reported",
    "counters_per_kernel": per,
    "command": f"tools/pmc_session.sh: rocprofv3 --pmc <one group per pass> -- python3 bench.py --config {cfg} "
               "--steps 2 --warmup 1 --legs '' --no-cpu-baseline --no-pcie --no-index --no-reader",
    "round": tag,
}
print(json.dumps(out, indent=1))
