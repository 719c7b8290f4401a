#!/usr/bin/env python3
"""rocprofv3 kernel-trace averages of one kernel split by bench.py pass:
warm-up, the uninstrumented wall-clock pass (K steps) and the HIP-event timing
pass (the last K launches).

    python tools/rocpd_passes.py gpurun_out/prof/run_results.db k_ecdsa_comb 50"""
import sqlite3
import statistics as st
import sys


def main(db, kern, k):
    c = sqlite3.connect(db)
    d = [(e - s) / 1e3 for n, s, e in c.execute("select name, start, end from kernels order by start") if kern in n]
    parts = {"all": d, "warm-up": d[:-2 * k], "wall-clock pass": d[-2 * k:-k], "timing-event pass": d[-k:]}
    for name, v in parts.items():
        if v:
            print(f"{name:18s} launches {len(v):4d}  mean {st.mean(v):9.2f} us  median {st.median(v):9.2f} us  "
                  f"max {max(v):9.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]))
