"""Summarise a tools/gpu_profile.sh run into profiles/ and profiles/pmc_traffic.json.

usage: python tools/pmc_summary.py <gpurun_out/prof_TAG> <profiles/rNN_TAG>

Writes <dst>/kernel_stats_<group>.csv (rocprofv3 --kernel-trace --stats
summary of each section group), <dst>/pmc_summary.json (per group, per-kernel
mean counters per launch) and updates profiles/pmc_traffic.json, which bench.py
reads for roofline.traffic / roofline.valu.  Counters are averaged over the
launches of each kernel in the PMC runs; tools/gpu_profile.sh runs the bench
sections in groups in which every decode kernel type serves ONE bench key, at
the bench's own batch sizes (no scaling of a smaller pass).

HBM-side traffic per launch = 2 * FETCH_SIZE + WRITE_SIZE (rocprofv3 reports
KiB; on gfx950 FETCH_SIZE counts 64 B per 128 B request -> doubled, as
MI355X_MICROARCH.md "HBM" prescribes; WRITE_SIZE as reported).  Infinity-cache
hits are counted too (the guide: they are not excluded), so this is traffic
beyond L2, an upper bound on DRAM bytes.
VALU: SQ_INSTS_VALU and its fp64 classes (ADD/MUL/FMA/TRANS _F64); bench.py
prices fp64 instructions at 4 SIMD cycles per wave64 and the rest at 2.
"""
import collections
import csv
import json
import os
import shutil
import sys

# bench.py pmc key -> (section group, kernel-name prefix, frames per launch in gpu_profile.sh)
KEYS = {
    "polar_scl_1024_l8": ("g1", "pl::polar_tree_kernel<10, 8, false, 3, 7, false, 4, 0>", 65536),
    "ldpc_bp_504": ("g1", "pl::ldpc_bp_grp_kernel<3, 6, 2, false", 65536),
    "polar_cascl_1024_l32": ("g1", "pl::polar_tree_kernel<10, 32, false, 3, 7, false, 4, 0>", 65536),
    "polar_scl_4096_l8": ("g1", "pl::polar_tree_kernel<12, 8, false, 4, 9, false, 4, 0>", 131072),
    "ldpc_ms_8192_noes": ("g1", "pl::ldpc_ms", 131072),
    "polar_scl_1024_l8_default": ("g2", "pl::polar_tree_kernel<10, 8, false, 3, 7, false, 4, 0>", 65536),
    "polar_sc_1024_default": ("g2", "pl::polar_tree_kernel<10, 1, true, 1, 5, false, 2, 0>", 65536),
    "polar_sc_256": ("g2", "pl::polar_tree_kernel<8, 1, true, 1, 3, false, 2, 0>", 100),
    "ldpc_ms_8192": ("g2", "pl::ldpc_ms", 131072),
    "ldpc_bp_504_valid": ("g2", "pl::ldpc_bp_grp_kernel<3, 6, 2, false", 65536),
}
PASSES = ("fetch", "write", "valu", "mix", "l2", "wait")
F64 = ("SQ_INSTS_VALU_ADD_F64", "SQ_INSTS_VALU_MUL_F64", "SQ_INSTS_VALU_FMA_F64", "SQ_INSTS_VALU_TRANS_F64")


def per_kernel(path):
    d = collections.defaultdict(list)
    if not os.path.exists(path):
        return {}
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        d[(name, r["Counter_Name"])].append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in d.items()}


def summarise(src):
    counters = {}
    for p in PASSES:
        for (name, cname), v in per_kernel(os.path.join(src, "pmc_" + p, "run_counter_collection.csv")).items():
            counters.setdefault(name, {})[cname] = v
    summ = {}
    for name, c in counters.items():
        s = dict(c)
        if "FETCH_SIZE" in c and "WRITE_SIZE" in c:
            s["hbm_bytes_per_launch"] = 2 * c["FETCH_SIZE"] * 1024 + c["WRITE_SIZE"] * 1024
        if all(k in c for k in F64):
            s["valu_fp64_per_launch"] = sum(c[k] for k in F64)
        hit, miss = c.get("TCC_HIT_sum"), c.get("TCC_MISS_sum")
        if hit is not None and miss is not None and hit + miss > 0:
            s["l2_hit_rate"] = hit / (hit + miss)
        wc = c.get("SQ_WAVE_CYCLES")
        if wc and "SQ_WAIT_ANY" in c:
            # SQ_WAIT_ANY + SQ_WAIT_INST_ANY + SQ_ACTIVE_INST_ANY ~ SQ_WAVE_CYCLES (MI355X_MICROARCH.md, PMC slots)
            s["wave_time_shares"] = {k: c[k] / wc for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY",
                                                            "SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_LDS",
                                                            "SQ_ACTIVE_INST_SCA", "SQ_WAIT_INST_LDS") if k in c}
        summ[name] = s
    return summ


def launches(path):
    """Per kernel from the rocprofv3 kernel trace: launches, mean over all of
    them (what run_kernel_stats.csv averages: the bench's warmup launches
    included) and over the bench's timed launches (the last 10 of the 12 that
    --steps 10 --warmup 2 makes; the last n-1 of a key capped by
    --extra-steps), the figure bench.py's HIP-event kernel_ms measures."""
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = r["Kernel_Name"].replace("void ", "").split("(")[0]
        d[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6)
    out = {}
    for name, t in d.items():
        timed = t[-10:] if len(t) > 10 else t[1:] or t
        out[name] = dict(launches=len(t), mean_ms_all=sum(t) / len(t), mean_ms_timed=sum(timed) / len(timed),
                         timed_launches=len(timed), ms=[round(x, 4) for x in t])
    return out


def main(src, dst):
    os.makedirs(dst, exist_ok=True)
    groups = sorted(g for g in os.listdir(src) if os.path.isdir(os.path.join(src, g, "trace")))
    allsumm = {}
    for g in groups:
        gs = os.path.join(src, g)
        shutil.copy(os.path.join(gs, "trace", "run_kernel_stats.csv"), os.path.join(dst, "kernel_stats_%s.csv" % g))
        json.dump(launches(os.path.join(gs, "trace", "run_kernel_trace.csv")),
                  open(os.path.join(dst, "kernel_launches_%s.json" % g), "w"), indent=1, sort_keys=True)
        if os.path.exists(os.path.join(gs, "bench_trace.json")):
            shutil.copy(os.path.join(gs, "bench_trace.json"), os.path.join(dst, "bench_trace_%s.json" % g))
        allsumm[g] = summarise(gs)
    json.dump(allsumm, open(os.path.join(dst, "pmc_summary.json"), "w"), indent=1, sort_keys=True)
    bid = os.path.join(src, "build_id.txt")  # the profiled libpolarldpc.so (tools/gpu_profile.sh)
    build = open(bid).read().strip() if os.path.exists(bid) else None
    tp = os.path.join(os.path.dirname(dst.rstrip("/")), "pmc_traffic.json")
    traffic = json.load(open(tp)) if os.path.exists(tp) else {}
    for key, (g, prefix, frames) in KEYS.items():
        for name, s in allsumm.get(g, {}).items():
            if name.startswith(prefix) and "hbm_bytes_per_launch" in s:
                t = dict(bytes_per_launch=s["hbm_bytes_per_launch"], frames=frames, kernel=name,
                         source=os.path.join(dst, "pmc_summary.json") + " [%s]" % g, build=build)
                if "SQ_INSTS_VALU" in s:
                    t["valu_per_launch"] = s["SQ_INSTS_VALU"]
                if "valu_fp64_per_launch" in s:
                    t["valu_fp64_per_launch"] = s["valu_fp64_per_launch"]
                if "l2_hit_rate" in s:
                    t["l2_hit_rate"] = s["l2_hit_rate"]
                if "wave_time_shares" in s:
                    t["wave_time_shares"] = s["wave_time_shares"]
                traffic[key] = t
    json.dump(traffic, open(tp, "w"), indent=1, sort_keys=True)
    for g, summ in allsumm.items():
        for name, s in sorted(summ.items()):
            if s.get("hbm_bytes_per_launch", 0) > 1e6:
                print("%s %-66s %9.3f GB/launch  VALU %.3g (f64 %.3g)  L2 hit %.2f" % (
                    g, name[:66], s["hbm_bytes_per_launch"] / 1e9, s.get("SQ_INSTS_VALU", 0),
                    s.get("valu_fp64_per_launch", 0), s.get("l2_hit_rate", float("nan"))))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
