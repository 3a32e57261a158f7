"""Print per-launch counter means for one kernel from a tools/gpu_pmc2.sh run.
usage: python tools/pmc_print.py gpurun_out/pmc2_TAG [kernel-substring]"""
import collections, csv, glob, os, sys
root = sys.argv[1]; sub = sys.argv[2] if len(sys.argv) > 2 else "polar_"
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(f)):
        if sub in r["Kernel_Name"]:
            d[r["Counter_Name"]].append(float(r["Counter_Value"]))
    for k, v in d.items():
        print("%-32s %14.4g  (x%d launches)" % (k, sum(v) / len(v), len(v)))
