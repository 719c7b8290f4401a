"""Summarise tools/pmc_passes.sh output: per-kernel mean counter values over
dispatches, plus derived VALU-busy and HBM bytes per launch (FETCH_SIZE doubled
for gfx950 wide reads, MI355X_MICROARCH.md HBM/rocprofv3 section)."""
from __future__ import annotations

import csv
import glob
import json
import os
import re
import sys
from collections import defaultdict


def short(name: str) -> str:
    for k in ("k_ecdsa_comb", "k_ecdsa_scalars", "k_ecdsa_wave", "k_sha256", "k_tab_", "k_len_"):
        if k in name:
            return k.lstrip("k_").rstrip("_")
    return name[:40]


def main(d: str):
    vals = defaultdict(lambda: defaultdict(list))
    geom = {}
    for f in glob.glob(os.path.join(d, "*", "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            vals[short(row["Kernel_Name"])][row["Counter_Name"]].append(float(row["Counter_Value"]))
            g = re.search(r"k_ecdsa_comb<(\d+), (\d+)>", row["Kernel_Name"])
            if g:
                geom[(int(g.group(1)), int(g.group(2)))] = 1
    out = {}
    for k, cs in vals.items():
        m = {c: sum(v) / len(v) for c, v in cs.items()}
        if "SQ_ACTIVE_INST_VALU" in m and "GRBM_GUI_ACTIVE" in m and m["GRBM_GUI_ACTIVE"]:
            # quad-cycle units; 4 SIMDs x 256 CUs
            m["valu_busy_frac"] = m["SQ_ACTIVE_INST_VALU"] * 4 / (1024 * m["GRBM_GUI_ACTIVE"])
        if "SQ_WAVE_CYCLES" in m and m["SQ_WAVE_CYCLES"]:
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in m:
                    m[c + "_frac"] = m[c] / m["SQ_WAVE_CYCLES"]
        if "FETCH_SIZE" in m or "WRITE_SIZE" in m:
            m["hbm_bytes_per_launch"] = 2 * 1024 * m.get("FETCH_SIZE", 0) + 1024 * m.get("WRITE_SIZE", 0)
        out[k] = m
    res = {"source": "rocprofv3 --pmc, separate passes (tools/pmc_passes.sh) over bench.py --steps 2 --warmup 1 "
                     "--no-extras; means over dispatches; FETCH_SIZE/WRITE_SIZE in KiB, FETCH doubled (gfx950)",
           "counters": out}
    for k, m in out.items():
        if k in ("ecdsa_comb", "ecdsa_scalars") and "hbm_bytes_per_launch" in m:
            e = {"hbm_bytes_per_launch": m["hbm_bytes_per_launch"]}
            if "SQ_INSTS_VALU" in m and m.get("SQ_WAVES"):
                e["valu_insts_per_wave"] = m["SQ_INSTS_VALU"] / m["SQ_WAVES"]
            if k == "ecdsa_comb" and len(geom) == 1:
                e["geometry"] = list(next(iter(geom)))  # bench.py uses the traffic only for this geometry
            res[k] = e
    json.dump(res, sys.stdout, indent=1)
    print()


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc")
