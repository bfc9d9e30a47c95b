"""Summarise rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes into profiles/<name>.json.

    python tools/pmc_summary.py <out.json> <workload> <fetch_counter_collection.csv> <write_counter_collection.csv> [--lib <librai_amd.so>]

Per kernel: median per-launch FETCH_SIZE and WRITE_SIZE (rocprofv3 reports KiB), and the
HBM traffic estimate used by bench.py's roofline.traffic:
    traffic_bytes = 2 * FETCH_SIZE * 1024 + WRITE_SIZE * 1024
(the x2 is MI355X_MICROARCH.md's gfx950 correction: FETCH_SIZE reports half the bytes of a
wide coalesced streaming read; it is calibrated for 16 B/lane loads only, so the estimate is
marked uncalibrated for other access widths).  Infinity-Cache hits are counted as fetches.
Each entry records lib_sha256, the sha256 of the librai_amd.so the passes ran (default: the in-tree
library); bench.py only reports a traffic figure whose lib_sha256 matches the library it loaded.
"""
import hashlib
import os
import csv
import json
import statistics
import sys
from collections import defaultdict


def per_kernel(path, counter):
    vals = defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] == counter:
            vals[r["Kernel_Name"]].append(float(r["Counter_Value"]))
    return vals


def main():
    out, workload, fetch_csv, write_csv = sys.argv[1:5]
    libp = sys.argv[sys.argv.index("--lib") + 1] if "--lib" in sys.argv else os.path.join(
        os.path.dirname(os.path.abspath(__file__)), "..", "rl-algo-impls_amd", "lib", "librai_amd.so")
    lib_sha = hashlib.sha256(open(libp, "rb").read()).hexdigest()
    f, w = per_kernel(fetch_csv, "FETCH_SIZE"), per_kernel(write_csv, "WRITE_SIZE")
    try:
        doc = json.load(open(out))
    except FileNotFoundError:
        doc = {}
    for k in sorted(set(f) & set(w)):
        fk, wk = statistics.median(f[k]), statistics.median(w[k])
        short = k.replace("(anonymous namespace)::", "").replace("void ", "").split("(")[0]
        doc.setdefault(workload, {})[short] = {
            "kernel": k, "launches": [len(f[k]), len(w[k])], "FETCH_SIZE_KiB_median": fk,
            "WRITE_SIZE_KiB_median": wk, "traffic_bytes_per_launch": int(2 * fk * 1024 + wk * 1024),
            "lib_sha256": lib_sha,
            "note": "traffic = 2*FETCH_SIZE + WRITE_SIZE (gfx950 FETCH correction; uncalibrated below 16 B/lane)"}
    json.dump(doc, open(out, "w"), indent=1, sort_keys=True)
    print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
