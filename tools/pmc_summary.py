"""Per-dispatch averages of rocprofv3 --pmc counters for one kernel (diagnostics).

Usage: python tools/pmc_summary.py <counter_collection.csv> [...] --kernel search_fast_kernel --out summary.json
Counters are summed over their dimensions within a dispatch, then averaged over the matching dispatches.
"""
import argparse
import csv
import json
from collections import defaultdict


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv", nargs="+")
    ap.add_argument("--kernel", default="search_fast_kernel")
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    per = defaultdict(lambda: defaultdict(float))
    names = {}
    for p in a.csv:
        with open(p, newline="") as f:
            for row in csv.DictReader(f):
                kn = row.get("Kernel_Name", "")
                if a.kernel not in kn:
                    continue
                d = (p, row.get("Dispatch_Id"))
                per[d][row["Counter_Name"]] += float(row["Counter_Value"])
                names[d] = kn
    by = defaultdict(list)
    for d, cs in per.items():
        for c, v in cs.items():
            by[c].append(v)
    out = {"kernels": sorted(set(names.values())), "dispatches": len(per),
           "per_dispatch": {c: sum(v) / len(v) for c, v in sorted(by.items())}}
    with open(a.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out["per_dispatch"], indent=1))


if __name__ == "__main__":
    main()
