"""Three host-buffer verifies of the config-4 batch (pinned inputs) for a
rocprofv3 --kernel-trace --memory-copy-trace timeline of the chunk pipeline."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tools"))
import synth  # noqa: E402
from simple_pbft_amd import Verifier  # noqa: E402

pub, H, S, K, ok = synth.config4(1 << 20, n_keys=100)
ver = Verifier()
ver.register_keys(pub)
pins = [ver.pinned(a) for a in (H, S, K)]
for _ in range(3):
    got = ver.verify_batch(*(p.a for p in pins))
assert (got == ok).all()
