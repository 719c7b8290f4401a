"""simple_pbft_amd -- MI355X-native batch verifier for simple_pbft's crypto hot path.

The product is ``libpbftv.so`` (gfx950 HIP kernels + the C ABI of
``include/pbftv.h``); :mod:`simple_pbft_amd.pbftv` is its ctypes binding and
:mod:`simple_pbft_amd.consensus` mirrors the reference's Go call sites
(utils.Hash, digest, State.verifyMsg, the message pools) on top of it.
"""
from .pbftv import (PBFTV_EDEVICE, PBFTV_EINVAL, PBFTV_ENODEV, PBFTV_ENOKEYS, PBFTV_ENOMEM, PBFTV_OK, PbftvError,
                    Verifier, bitmap_to_bool, lib)

__all__ = ["Verifier", "PbftvError", "lib", "bitmap_to_bool", "PBFTV_OK", "PBFTV_EINVAL", "PBFTV_ENODEV",
           "PBFTV_EDEVICE", "PBFTV_ENOMEM", "PBFTV_ENOKEYS"]
