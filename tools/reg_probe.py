"""Key-registration cost (SURVEY.md §8(d) row f): wall time
of pbftv_register_keys for 100 keys (G table + 100 key tables) with the
library's per-phase trace (PBFTV_TRACE, read through bench.register_with_phases),
in the situations a node meets:
  first        the first registration of the process (a fresh context)
  again        the same key set again in that context (tables rebuilt in place)
  reopened     pbftv_close, then a new context registers: the 234 GB the old
               one freed is allocated again at once
plus pbftv_add_keys of one key and pbftv_set_key.  Run it twice in a row to
see a process that starts right after another one freed its tables.  One
JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
os.environ.setdefault("PBFTV_TRACE", "1")
import bench  # noqa: E402
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K, ok = synth.config4(4096, n_keys=101, pool=4096)
out = {}
t = time.perf_counter()
ver = Verifier(device_mask=1)
out["open_s"] = time.perf_counter() - t
for label in ("first", "again"):
    _, wall, ph = bench.register_with_phases(ver, pub[:100])
    out[label] = {"wall_s": wall, "phases_ms": ph}
out["geometry"] = list(ver.table_config())
t = time.perf_counter()
ver.add_keys(pub[100:101])
out["add_1_key_s"] = time.perf_counter() - t
t = time.perf_counter()
ver.set_key(3, pub[3])
out["set_1_key_s"] = time.perf_counter() - t
out["check"] = bool((ver.verify_batch(H, S, K) == ok).all())
t = time.perf_counter()
ver.close()
out["close_s"] = time.perf_counter() - t
ver = Verifier(device_mask=1)
_, wall, ph = bench.register_with_phases(ver, pub[:100])
out["reopened"] = {"wall_s": wall, "phases_ms": ph}
out["check_reopened"] = bool((ver.verify_batch(H, S, K) == (ok & (K < 100))).all())  # key 100 not registered
ver.close()
print(json.dumps(out))
