"""Summarise tools/pmc_passes.sh output into per-kernel counter means and the
derived figures the roofline claims rest on:

  cycles           = GRBM_GUI_ACTIVE / 8   (rocprofv3 sums GRBM over the 8 XCDs,
                                             MI355X_MICROARCH.md "DVFS give-back")
  valu_insts_per_wave = SQ_INSTS_VALU / SQ_WAVES
  valu_busy_frac   = SQ_ACTIVE_INST_VALU / (256 CUs x cycles)   -- rocprofv3's
                     VALUBusy with the XCD sum undone; it prices every VALU
                     instruction at 4 cycles on one of the CU's 4 SIMDs
  valu_issue_frac  = (SQ_INSTS_VALU_INT64 x c64 + (SQ_INSTS_VALU - INT64) x c32)
                     / (1024 SIMDs x cycles), with the issue costs measured by
                     tools/mad_issue_bench.hip at 4 waves/SIMD (c64: v_mad_u64_u32 /
                     v_mad_i64_i32 / 64-bit shifts and adds; c32: 32-bit VALU)
  hbm_bytes_per_launch = f x FETCH_SIZE + WRITE_SIZE (KiB; f = 2 for coalesced
                     wide reads, MI355X_MICROARCH.md HBM/rocprofv3 section; f = 1
                     for the comb, whose traffic is random 64-B table gathers,
                     which FETCH_SIZE counts at their size: tools/gather_calib.hip
                     measured 1.12x the gathered bytes for 64-B gathers and 0.50x
                     for 128-B ones, profiles/r02_gather_calib.txt)
  kernel_ms        = mean dispatch duration in the (profiled) kernel trace

    python tools/pmc_summary.py gpurun_out/pmc [issue-cost file] > profiles/rNN_pmc.json
"""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict

# measured issue costs (SIMD-cycles per wave-instruction, 4 waves/SIMD,
# profiles/r02_microbench_mad_issue.txt)
C64 = 4.5
C32 = 2.95
SIMDS = 1024
CUS = 256


def short(name: str) -> str:
    m = re.search(r"k_ecdsa_comb<(\d+), (\d+)>", name)
    if m:
        return "ecdsa_comb"
    for k in ("k_ecdsa_scalars", "k_ecdsa_wave", "k_sha256", "k_key_hist", "k_key_scatter", "k_key_scan",
              "k_pack_bits", "k_len_", "k_gojson", "k_tab_entries", "k_tab_small", "k_tab_bases"):
        if k in name:
            return k[2:].rstrip("_")
    return name[:40]


def issue_costs(path):
    """c64 / c32 from a mad_issue_bench listing (4 waves/SIMD rows), if given."""
    if not path or not os.path.exists(path):
        return C64, C32
    c64, c32 = [], []
    for line in open(path):
        m = re.match(r"(.+?)\s+waves/SIMD=4\s+([\d.]+)", line)
        if not m:
            continue
        name, v = m.group(1).strip(), float(m.group(2))
        if name.startswith(("mad_u64 16 indep", "mad_i64_i32", "lshl_add_u64")):
            c64.append(v)
        elif name.startswith(("add_u32", "not_b32")):
            c32.append(v)
    return (sum(c64) / len(c64) if c64 else C64), (sum(c32) / len(c32) if c32 else C32)


def main(d: str, costs: str | None):
    c64, c32 = issue_costs(costs)
    vals = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(list)
    geom = set()
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
            g = re.search(r"k_ecdsa_comb<(\d+), (\d+)>", row["Kernel_Name"])
            if g:
                geom.add((int(g.group(1)), int(g.group(2))))
    for f in glob.glob(os.path.join(d, "*", "**", "*kernel_trace.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            dur[short(row["Kernel_Name"])].append((int(row["End_Timestamp"]) - int(row["Start_Timestamp"])) * 1e-6)
    out = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        e = {"counters": m}
        if dur.get(k):
            e["kernel_ms"] = sum(dur[k]) / len(dur[k])
        cyc = m.get("GRBM_GUI_ACTIVE", 0) / 8
        if cyc:
            e["cycles"] = cyc
            if "SQ_ACTIVE_INST_VALU" in m:
                e["valu_busy_frac"] = m["SQ_ACTIVE_INST_VALU"] / (CUS * cyc)
            if "SQ_INSTS_VALU" in m and "SQ_INSTS_VALU_INT64" in m:
                i64 = m["SQ_INSTS_VALU_INT64"]
                e["valu_issue_frac"] = (i64 * c64 + (m["SQ_INSTS_VALU"] - i64) * c32) / (SIMDS * cyc)
                e["int64_share"] = i64 / m["SQ_INSTS_VALU"] if m["SQ_INSTS_VALU"] else 0.0
            if e.get("kernel_ms"):
                e["clock_ghz"] = cyc / (e["kernel_ms"] * 1e-3) / 1e9
        if m.get("SQ_WAVES"):
            if "SQ_INSTS_VALU" in m:
                e["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
        if m.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    e[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            f = 1 if k == "ecdsa_comb" else 2  # 64-B random gathers: counted at size (gather_calib)
            e["hbm_bytes_per_launch"] = f * 1024 * m.get("FETCH_SIZE", 0) + 1024 * m.get("WRITE_SIZE", 0)
            e["fetch_factor"] = f
        if k == "ecdsa_comb" and len(geom) == 1:
            e["geometry"] = list(next(iter(geom)))  # bench.py uses these figures only for this geometry
        out[k] = e
    res = {"source": "rocprofv3 --pmc, separate passes (tools/pmc_passes.sh) over tools/pmc_workload.py "
                     "(config-4 verify, config-5 digests, one n=4 certificate); means over dispatches; "
                     "FETCH_SIZE/WRITE_SIZE in KiB, FETCH doubled (gfx950 wide reads) except for the comb's "
                     "64-B gathers (fetch_factor 1, tools/gather_calib.hip); GRBM_GUI_ACTIVE / 8 XCDs",
           "issue_costs": {"c64": c64, "c32": c32, "from": costs or "defaults"},
           "kernels": out}
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc", sys.argv[2] if len(sys.argv) > 2 else None)
