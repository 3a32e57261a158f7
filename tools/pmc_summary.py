"""Summarise a tools/gpu_full.sh (or gpu_prof.sh) run into profiles/.

usage: python tools/pmc_summary.py <gpurun_out/full_TAG> <profiles/rNN_TAG>

Writes <dst>/kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
<dst>/pmc_summary.json (per-kernel mean FETCH_SIZE / WRITE_SIZE per launch) and
updates profiles/pmc_traffic.json, which bench.py reads for roofline.traffic.

SQ_INSTS_VALU (wave-level VALU instructions) per launch is recorded too when the
pmc_valu pass exists.
HBM traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (rocprofv3 reports KiB;
FETCH_SIZE counts 64 B per 128 B request on gfx950 -> doubled, as
MI355X_MICROARCH.md "HBM" prescribes; WRITE_SIZE is taken as reported).
"""
import csv
import collections
import json
import os
import shutil
import sys

KEYS = {  # bench.py traffic key -> kernel-name prefix
    "polar_scl_1024_l8": "void pl::polar_tree_kernel<10, 8, false, 3, 7, false, 4>",
    "ldpc_bp_504": "void pl::ldpc_reg_kernel<0, 3, 6, 2>",
}


def per_kernel(path):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        d[(r["Kernel_Name"], r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats.csv"))
    for f in ("bench.json", "bench_trace.json"):
        if os.path.exists(os.path.join(src, f)):
            shutil.copy(os.path.join(src, f), os.path.join(dst, f))
    fetch = per_kernel(os.path.join(src, "pmc_fetch", "run_counter_collection.csv"))
    write = per_kernel(os.path.join(src, "pmc_write", "run_counter_collection.csv"))
    vp = os.path.join(src, "pmc_valu", "run_counter_collection.csv")
    valu = per_kernel(vp) if os.path.exists(vp) else {}
    summ = {}
    for (name, _), v in fetch.items():
        w = write.get((name, "WRITE_SIZE"), 0.0)
        summ[name] = dict(fetch_size_kib=v, write_size_kib=w,
                          hbm_bytes_per_launch=2 * v * 1024 + w * 1024)
        if (name, "SQ_INSTS_VALU") in valu:
            summ[name]["valu_instr_per_launch"] = valu[(name, "SQ_INSTS_VALU")]
            summ[name]["waves_per_launch"] = valu.get((name, "SQ_WAVES"))
    json.dump(summ, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1)
    tp = os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_traffic.json")
    traffic = json.load(open(tp)) if os.path.exists(tp) else {}
    for key, prefix in KEYS.items():
        for name, s in summ.items():
            if name.startswith(prefix):
                traffic[key] = dict(bytes_per_launch=s["hbm_bytes_per_launch"], source=os.path.join(dst, "pmc_summary.json"),
                                    kernel=name.split("(")[0])
                if "valu_instr_per_launch" in s:
                    traffic[key]["valu_instr_per_launch"] = s["valu_instr_per_launch"]
    json.dump(traffic, open(tp, "w"), indent=1)
    for name, s in summ.items():
        if s["hbm_bytes_per_launch"] > 1e6:
            print("%-60s %10.3f GB/launch" % (name[:60], s["hbm_bytes_per_launch"] / 1e9))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
