"""MI355X-native STFT-gate-OLA engine with the host API of the Tomatis processor.

Product path: host Python (this package) -> C ABI ``libtomatis_hip.so``
(hand-written gfx950 HIP kernels).  See DESIGN.md / INTEGRATION.md.
"""
from ._lib import TomatisLibraryError, lib  # noqa: F401

__version__ = "0.1.0"
