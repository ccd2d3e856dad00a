"""Summarise rocprofv3 --pmc counter CSVs of benchmarks/kernel_probe.py runs (ddpx kernels only)."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def summarise(root):
    out = {}
    for case_dir in sorted(glob.glob(os.path.join(root, "*"))):
        case = os.path.basename(case_dir)
        agg = defaultdict(lambda: defaultdict(list))
        for f in glob.glob(os.path.join(case_dir, "*", "*counter_collection.csv")):
            for r in csv.DictReader(open(f)):
                name = r["Kernel_Name"]
                if "ddpx" not in name:
                    continue
                key = name.split("(")[0][-70:]
                agg[key][r["Counter_Name"]].append(float(r["Counter_Value"]))
                agg[key]["_dur_ns"].append(float(r["End_Timestamp"]) - float(r["Start_Timestamp"]))
                agg[key]["_vgpr"] = [float(r["VGPR_Count"])]
                agg[key]["_agpr"] = [float(r["Accum_VGPR_Count"])]
        out[case] = {k: {c: sum(v) / len(v) for c, v in d.items()} for k, d in agg.items()}
    return out


if __name__ == "__main__":
    res = {}
    for root in sys.argv[1:]:
        for case, d in summarise(root).items():
            res.setdefault(case, {})
            for k, cs in d.items():
                res[case].setdefault(k, {}).update(cs)
    print(json.dumps(res, indent=1))
