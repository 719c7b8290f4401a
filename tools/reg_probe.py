"""Key-registration cost (SURVEY.md §8(d) row f / VERDICT r01 item 9): wall
time of pbftv_register_keys for 100 keys (G table + 100 key tables), a second
registration (G table kept), pbftv_add_keys of one key and pbftv_set_key, with
the library's phase trace (PBFTV_TRACE=1) on stderr.  One JSON line."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K, ok = synth.config4(4096, n_keys=101, pool=4096)
ver = Verifier()
out = {}
t = time.perf_counter()
ver.register_keys(pub[:100])
out["register_100_first_s"] = time.perf_counter() - t
out["geometry"] = list(ver.table_config())
t = time.perf_counter()
ver.register_keys(pub[:100])
out["register_100_again_s"] = time.perf_counter() - t
t = time.perf_counter()
ver.add_keys(pub[100:101])
out["add_1_key_s"] = time.perf_counter() - t
t = time.perf_counter()
ver.set_key(3, pub[3])
out["set_1_key_s"] = time.perf_counter() - t
got = ver.verify_batch(H, S, K)
out["check"] = bool((got == ok).all())
print(json.dumps(out))
