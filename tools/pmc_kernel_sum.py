"""Mean per-dispatch PMC counters of the kernels whose name matches a pattern,
from rocprofv3 --pmc CSV directories (tools/ldpc_pmc.sh output).

usage: python tools/pmc_kernel_sum.py <pattern> <dir> [<dir> ...]  -> JSON on stdout"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def load(pattern, dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            for r in csv.DictReader(open(f)):
                if pattern in r["Kernel_Name"]:
                    acc[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


if __name__ == "__main__":
    print(json.dumps(load(sys.argv[1], sys.argv[2:]), indent=1))
