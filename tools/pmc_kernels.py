"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (run on the GPU box, so the raw
per-dispatch CSV — hundreds of MB for a training update — never has to travel back).

    python tools/pmc_kernels.py <counter_collection.csv> <out.json> [--delete]

Per kernel name: dispatches, the sum of every collected counter.  When SQ_VALU_MFMA_BUSY_CYCLES and
GRBM_GUI_ACTIVE were collected, mfma_busy_frac = MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs * 4 SIMDs)
(the gfx94x MfmaUtil formula; rocprofv3 sums GRBM_GUI_ACTIVE over the 8 XCDs, MI355X_MICROARCH.md).
"""
import csv
import json
import os
import sys
from collections import defaultdict


def main():
    path, out = sys.argv[1], sys.argv[2]
    sums = defaultdict(lambda: defaultdict(float))
    dispatches = defaultdict(set)
    with open(path) as f:
        for r in csv.DictReader(f):
            k = r["Kernel_Name"]
            sums[k][r["Counter_Name"]] += float(r["Counter_Value"])
            dispatches[k].add(r["Dispatch_Id"])
    doc = {}
    for k, c in sums.items():
        e = {"dispatches": len(dispatches[k]), **{n: v for n, v in c.items()}}
        if "SQ_VALU_MFMA_BUSY_CYCLES" in c and c.get("GRBM_GUI_ACTIVE"):
            e["mfma_busy_frac"] = c["SQ_VALU_MFMA_BUSY_CYCLES"] / (c["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
        doc[k] = e
    tot = defaultdict(float)
    for e in doc.values():
        for n, v in e.items():
            if n not in ("dispatches", "mfma_busy_frac"):
                tot[n] += v
    summary = {"_total": dict(tot), "kernels": dict(sorted(doc.items(), key=lambda kv: -kv[1].get("GRBM_GUI_ACTIVE", 0)))}
    if "SQ_VALU_MFMA_BUSY_CYCLES" in tot and tot.get("GRBM_GUI_ACTIVE"):
        summary["_total"]["mfma_busy_frac"] = tot["SQ_VALU_MFMA_BUSY_CYCLES"] / (tot["GRBM_GUI_ACTIVE"] / 8 * 256 * 4)
    json.dump(summary, open(out, "w"), indent=1)
    if "--delete" in sys.argv:
        os.remove(path)
    print(f"{len(doc)} kernels -> {out}")


if __name__ == "__main__":
    main()
