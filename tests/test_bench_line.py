"""The driver keeps only the last ~8 KB of bench.py's stdout (VERDICT r03:
BENCH_r03 parsed null because the full line was 24 KB).  The stdout line is
built by bench.compact_line; this checks it on the round-3 payload."""
import json
import os

import bench

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _payload():
    with open(os.path.join(ROOT, "profiles", "r03_j", "bench.json")) as f:
        return json.load(f)


def test_compact_line_fits_driver_tail():
    full = _payload()
    line = bench.compact_line(full, "gpurun_out/bench_detail.json")
    s = json.dumps(line)
    assert len(s) <= bench.MAX_LINE, len(s)
    assert "\n" not in s
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "dtype", "config",
              "roofline", "cpu_baseline", "higher_is_better", "scaling", "vs_baseline", "data"):
        assert k in line, k
    r = line["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic", "kernel", "kernel_ms"):
        assert k in r and r[k] is not None, k
    c = line["cpu_baseline"]
    for k in ("value", "cores", "kind", "mismatches"):
        assert k in c and c[k] is not None, k
    assert abs(line["value"] - full["value"]) / full["value"] < 1e-5
    # every secondary key keeps a compact summary with its roofline fraction
    for name in ("ldpc", "cascl_l32", "end_to_end", "default_frozen_set", "polar_sc_default", "config0_sc_256",
                 "long_block.polar_4096_l8", "long_block.ldpc_8192_ms20",
                 "long_block.ldpc_8192_ms20_no_early_stop", "ldpc.valid_codewords"):
        assert name in line["keys"], name
        assert line["keys"][name]["value"] is not None
    for name in ("ldpc", "cascl_l32", "long_block.polar_4096_l8"):
        assert line["keys"][name]["frac"] is not None
    assert json.loads(s) == line


def test_compact_line_survives_extra_ranks():
    """An 8-rank line (per-rank times) stays under the limit too."""
    full = _payload()
    full["rank_ms_per_step"] = [6.123456789] * 8
    for v in full.values():
        if isinstance(v, dict) and "rank_ms_per_step" in v:
            v["rank_ms_per_step"] = [6.123456789] * 8
    assert len(json.dumps(bench.compact_line(full, "x"))) <= bench.MAX_LINE
