"""Timeline of the last host-buffer verify in a rocprofv3 --kernel-trace
--memory-copy-trace CSV run (tools/host_path_trace.py): every kernel and copy
with start/end relative to the call's first copy, and the copy engine's idle
gaps.

    python tools/host_path_timeline.py gpurun_out/hpt/prof [events]
"""
import csv
import os
import sys


def main():
    d = sys.argv[1]
    last = int(sys.argv[2]) if len(sys.argv) > 2 else 80
    ev = []
    for r in csv.DictReader(open(os.path.join(d, "run_kernel_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "K", r["Kernel_Name"][:48]))
    for r in csv.DictReader(open(os.path.join(d, "run_memory_copy_trace.csv"))):
        ev.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), "C", r["Direction"] + " " + r.get("Size", "")))
    ev.sort()
    ev = ev[-last:]
    # start the window at the first H2D copy of the last call
    first = next(i for i, e in enumerate(ev) if e[2] == "C" and "HOST_TO_DEVICE" in e[3])
    ev = ev[first:]
    t0 = ev[0][0]
    prev_c = None
    gaps = []
    for s, e, t, n in ev:
        gap = ""
        if t == "C":
            if prev_c is not None:
                gaps.append(s - prev_c)
                gap = f"  copy gap {(s - prev_c) / 1000:6.1f}"
            prev_c = e
        print(f"{(s - t0) / 1000:9.1f} {(e - t0) / 1000:9.1f} {(e - s) / 1000:8.1f} {t} {n}{gap}")
    copies = [e for e in ev if e[2] == "C"]
    busy = sum(e - s for s, e, t, n in copies)
    span = ev[-1][1] - t0
    print(f"span {span / 1000:.1f} us, copy busy {busy / 1000:.1f} us, copy gaps {sum(gaps) / 1000:.1f} us "
          f"over {len(gaps)} gaps")


if __name__ == "__main__":
    main()
