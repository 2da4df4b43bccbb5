"""Mean per dispatch of each PMC counter, per kernel, from rocprofv3
counter_collection CSVs (one row per counter per dispatch).
    python scripts/pmc_summary.py FILE... [--kernel SUBSTR] [--json OUT]"""
import csv
import json
import sys
from collections import defaultdict


def summarise(path, filt):
    acc = defaultdict(lambda: defaultdict(list))
    res = {}
    for row in csv.DictReader(open(path)):
        k = row.get("Kernel_Name", "")
        if filt in k:
            acc[k][row["Counter_Name"]].append(float(row["Counter_Value"]))
            res.setdefault(k, {"vgpr": row["VGPR_Count"], "agpr": row["Accum_VGPR_Count"],
                               "lds": row["LDS_Block_Size"], "grid": row["Grid_Size"]})
    return {k: {"resources": res[k], "per_dispatch_mean": {c: sum(v) / len(v) for c, v in cs.items()}}
            for k, cs in acc.items()}


def main():
    args = sys.argv[1:]
    filt = args[args.index("--kernel") + 1] if "--kernel" in args else "analysis"
    out = args[args.index("--json") + 1] if "--json" in args else None
    files = [a for i, a in enumerate(args) if not a.startswith("--") and (i == 0 or args[i - 1] not in ("--kernel", "--json"))]
    allres = {}
    for f in files:
        for k, r in summarise(f, filt).items():
            allres.setdefault(k, {"resources": r["resources"], "per_dispatch_mean": {}})
            allres[k]["per_dispatch_mean"].update(r["per_dispatch_mean"])
    for k, r in allres.items():
        print(k[:100], r["resources"])
        for c, v in sorted(r["per_dispatch_mean"].items()):
            print(f"   {c:32s} {v:.5g}")
    if out:
        json.dump(allres, open(out, "w"), indent=1)


if __name__ == "__main__":
    main()
