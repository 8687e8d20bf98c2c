"""ctypes binding of the gfx950 C-ABI library ``libtomatis_hip.so``.

The library is the product: there is no CPU fallback.  ``lib()`` raises
``TomatisLibraryError`` when the shared object is missing or fails to load, and
every entry point's int status is turned into an exception by ``check``.

``torch`` is imported (when available) *before* the library is loaded so that
the process holds a single HIP runtime: torch's bundled ``libamdhip64.so`` has
the same SONAME (``libamdhip64.so.7``) as the one the library links against.
"""
from __future__ import annotations

import ctypes as C
import os

LIB_NAME = "libtomatis_hip.so"
ABI_VERSION = 11  # include/tomatis_hip.h TOMATIS_ABI_VERSION
GATE_SEGMENT = 1024      # TOMATIS_GATE_SEGMENT
GATE_NONE = -536870912   # TOMATIS_GATE_NONE
ERR_LIMITER_WAIT = 1     # TOMATIS_ERR_LIMITER_WAIT
ERR_PAIR_BARRIER = 2     # TOMATIS_ERR_PAIR_BARRIER
ERR_GATE_CARRY = 4       # TOMATIS_ERR_GATE_CARRY
E_UNSUPPORTED = -2       # TOMATIS_E_UNSUPPORTED
OPT_FUSE_LIMITER = 1     # TOMATIS_OPT_FUSE_LIMITER
OPT_LIMITER_SPIN = 2     # TOMATIS_OPT_LIMITER_SPIN
OPT_MINHOLD_SERIAL = 3   # TOMATIS_OPT_MINHOLD_SERIAL
# development overrides (TOMATIS_DEV_*: tests and A/B experiments only)
DEV_KEYS = dict(FAST_LOOP=1, RUN_ROUNDS=2, RUN_FRAMES=3, LEVELS_LEGACY=4, GATE_TF=5, MH_PARTS=6,
                FORCE_LDS=7, P64=8, ALPHA_SEQ=9, GAIN_LDS=10, FUSE_LIMITER=11, WG=12,
                SLOTS=13, FUSED_LEVELS=14, FUSED_4096=15)
HERE = os.path.dirname(os.path.abspath(__file__))

F32, F64 = 0, 1
NORM_EPS, NORM_MAX = 0, 1


class TomatisLibraryError(RuntimeError):
    pass


class TomatisStream(C.Structure):
    """Mirror of ``TomatisStream`` in include/tomatis_hip.h."""
    _fields_ = [
        ("in_off", C.c_int64), ("out_off", C.c_int64), ("n", C.c_int64),
        ("first_start", C.c_int64), ("n_frames", C.c_int64),
        ("out_begin", C.c_int64), ("out_len", C.c_int64),
        ("chunk_first", C.c_int64), ("chunk_len", C.c_int64),
        ("n_chunks", C.c_int32), ("in_scale", C.c_float), ("out_scale", C.c_float),
        ("on_bits", C.c_uint32), ("off_bits", C.c_uint32),
        ("on_exc", C.c_uint32 * 4), ("off_exc", C.c_uint32 * 4),
        ("n_on_exc", C.c_int32), ("n_off_exc", C.c_int32),
        ("t_on", C.c_double), ("t_off", C.c_double),
        ("frame_base", C.c_int64), ("chunk_base", C.c_int32), ("_pad", C.c_int32),
    ]


class TomatisGateCand(C.Structure):
    """Mirror of ``TomatisGateCand`` in include/tomatis_hip.h (24 bytes)."""
    _fields_ = [("level_row", C.c_int32), ("t_on", C.c_float), ("t_off", C.c_float),
                ("pad_", C.c_int32), ("up_delay", C.c_int64)]


GATE_CAND_DTYPE = [("level_row", "<i4"), ("t_on", "<f4"), ("t_off", "<f4"), ("pad_", "<i4"),
                   ("up_delay", "<i8")]


class TomatisPlanDesc(C.Structure):
    _fields_ = [
        ("n_fft", C.c_int32), ("hop", C.c_int32), ("ch", C.c_int32),
        ("norm_mode", C.c_int32), ("up_delay_frames", C.c_int32),
        ("min_hold_frames", C.c_int32), ("xfade_frames", C.c_int32),
        ("alpha_mode", C.c_int32),
    ]


_P = C.c_void_p
_SIGS = {
    "tomatis_abi_version": (C.c_int, []),
    "tomatis_status_string": (C.c_char_p, [C.c_int]),
    "tomatis_plan_create": (C.c_int, [C.POINTER(_P), C.POINTER(TomatisPlanDesc),
                                      C.POINTER(C.c_float), C.POINTER(TomatisStream),
                                      C.c_int32]),
    "tomatis_plan_destroy": (C.c_int, [_P]),
    "tomatis_plan_total_frames": (C.c_int64, [_P]),
    "tomatis_plan_total_chunks": (C.c_int32, [_P]),
    "tomatis_plan_update_streams": (C.c_int, [_P, C.POINTER(TomatisStream), _P]),
    "tomatis_levels": (C.c_int, [_P, _P, _P, C.c_int32, _P]),
    "tomatis_gate_std": (C.c_int, [_P, _P, _P, _P, _P, _P]),
    "tomatis_plan_gate_segments": (C.c_int32, [_P]),
    "tomatis_gate_segment_sums": (C.c_int, [_P, _P, _P, _P]),
    "tomatis_gate_std_carry": (C.c_int, [_P, _P, _P, _P, _P, _P]),
    "tomatis_level_stats": (C.c_int, [_P, _P, _P, _P]),
    "tomatis_minhold_bisect": (C.c_int, [_P, _P, _P, C.c_double, C.c_double, _P, _P, _P,
                                         _P, _P]),
    "tomatis_stft_ola": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, _P, _P]),
    "tomatis_apply_limiter": (C.c_int, [_P, _P, _P, C.c_float, _P]),
    "tomatis_stft_ola_limited": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, _P, C.c_float, _P]),
    "tomatis_stft_ola_limited_edges": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, _P, C.c_float,
                                                 C.c_int32, _P]),
    "tomatis_apply_limiter_edges": (C.c_int, [_P, _P, _P, C.c_float, C.c_int32, _P]),
    "tomatis_stft_ola_gated": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, C.c_float, _P, _P, _P]),
    "tomatis_gate_lookback": (C.c_int, [_P, _P, _P]),
    "tomatis_plan_set_gate_alpha": (C.c_int, [_P, _P]),
    "tomatis_flacd_workspace_bytes": (C.c_int64, [C.c_int64, C.c_int32]),
    "tomatis_flacd_plan": (C.c_int, [_P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P]),
    "tomatis_flacd_write": (C.c_int, [_P, C.c_int64, C.c_int32, C.c_int32, _P, _P, _P, _P]),
    "tomatis_flacd_find": (C.c_int, [_P, C.c_int64, C.c_int64, C.c_int32, C.c_int32, _P,
                                     C.c_int32, _P, _P]),
    "tomatis_flacd_scan": (C.c_int, [_P, C.c_int64, _P, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_int64, _P, _P]),
    "tomatis_flacd_decode": (C.c_int, [_P, C.c_int64, _P, C.c_int32, C.c_int32, C.c_int32,
                                       C.c_int64, _P, C.c_int64, _P, _P]),
    "tomatis_stft_ola_gated_after_lookback": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, C.c_float,
                                                        _P, _P, _P]),
    "tomatis_stft_ola_gated_pipelined": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, C.c_float,
                                                   _P, _P, _P, _P, _P]),
    "tomatis_stft_ola_pipelined": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, _P, C.c_float,
                                             _P, _P, _P]),
    "tomatis_stft_ola_gated_pipelined_after": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, C.c_float,
                                                         _P, _P, _P, _P, _P, _P]),
    "tomatis_stft_ola_pipelined_after": (C.c_int, [_P, _P, _P, C.c_int32, _P, _P, _P, C.c_float,
                                                   _P, _P, _P, _P]),
    "tomatis_copy_probe": (C.c_int, [_P, _P, C.c_int64, _P]),
    "tomatis_ts_summary": (C.c_int, [_P, _P, C.c_int32, C.c_int32, _P, _P]),
    "tomatis_ts_gate": (C.c_int, [_P, _P, _P, C.c_int32, C.c_int32, _P, _P, _P]),
    "tomatis_plan_error": (C.c_int, [_P, _P]),
    "tomatis_plan_error_bits": (C.c_int, [_P, C.POINTER(C.c_uint32), C.c_int32, _P]),
    "tomatis_plan_set_option": (C.c_int, [_P, C.c_int32, C.c_int64]),
    "tomatis_set_dev_option": (C.c_int, [C.c_int32, C.c_int32]),
    "tomatis_get_dev_option": (C.c_int32, [C.c_int32]),
    "tomatis_absmax": (C.c_int, [_P, C.c_int64, _P, _P]),
    "tomatis_absmax_streams": (C.c_int, [_P, _P, _P, _P]),
    "tomatis_scale_copy": (C.c_int, [_P, _P, C.c_int64, C.c_float, _P]),
    "tomatis_synth_fill": (C.c_int, [_P, C.c_int64, C.c_int32, C.c_int32, C.c_uint32,
                                     C.c_int64, _P]),
    "tomatis_pcm_to_float": (C.c_int, [_P, C.c_int64, C.c_int32, _P, _P]),
    "tomatis_float_to_pcm": (C.c_int, [_P, C.c_int64, C.c_int32, _P, _P]),
    # analysis spectra
    "tomatis_an_frame_r": (C.c_int, [_P, C.c_int64, C.c_int32, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_float, _P, _P]),
    "tomatis_an_select": (C.c_int, [_P, C.c_int32, C.c_uint32, C.POINTER(C.c_uint32), C.c_int32,
                                    C.c_int32, _P, C.c_int32, _P, _P, _P]),
    "tomatis_an_spectra": (C.c_int, [_P, _P, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                     C.c_int32, C.c_int32, C.c_float, _P, _P, _P]),
    "tomatis_an_frame_mean": (C.c_int, [_P, C.c_int32, C.c_int32, _P, _P]),
    "tomatis_an_median_work_words": (C.c_int64, [C.c_int32]),
    "tomatis_an_frame_median": (C.c_int, [_P, C.c_int32, C.c_int32, _P, C.c_int32, _P, _P, _P]),
    # gate calibration
    "tomatis_an_band_energy": (C.c_int, [_P, C.c_int64, C.c_int32, C.c_int32, C.c_int32,
                                         C.c_int32, C.c_int32, C.c_int32, _P, _P, _P]),
    "tomatis_cal_gate_grid": (C.c_int, [_P, C.c_int32, _P, _P, _P, C.c_int32, _P, _P, _P]),
}
EXPORTS = tuple(_SIGS)

_LIB = None


def lib_path() -> str:
    return os.environ.get("TOMATIS_HIP_LIB", os.path.join(HERE, LIB_NAME))


def lib():
    """Load (once) and return the ctypes handle; raise if it cannot be loaded."""
    global _LIB
    if _LIB is not None:
        return _LIB
    path = lib_path()
    if not os.path.exists(path):
        raise TomatisLibraryError(
            f"{path} not found: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            " (hipcc --offload-arch=gfx950). There is no CPU fallback.")
    try:
        import torch  # noqa: F401  (single HIP runtime, see module docstring)
    except Exception:  # pragma: no cover - torch is part of the image
        pass
    try:
        h = C.CDLL(path, mode=C.RTLD_GLOBAL)
    except OSError as e:
        raise TomatisLibraryError(f"cannot load {path}: {e}") from e
    for name, (res, args) in _SIGS.items():
        fn = getattr(h, name)
        fn.restype = res
        fn.argtypes = args
    if h.tomatis_abi_version() != ABI_VERSION:
        raise TomatisLibraryError("ABI version mismatch")
    _LIB = h
    return h


def check(rc: int, what: str = "") -> None:
    if rc != 0:
        msg = lib().tomatis_status_string(rc).decode()
        raise RuntimeError(f"{what or 'tomatis'} failed: {msg} (status {rc})")


def ptr(t) -> C.c_void_p:
    """Device pointer of a torch tensor (or None -> NULL)."""
    if t is None:
        return C.c_void_p(0)
    return C.c_void_p(t.data_ptr())


def stream_handle(device=None) -> C.c_void_p:
    import torch
    return C.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def set_dev_option(name: str, value: int):
    """tomatis_set_dev_option(TOMATIS_DEV_<name>, value); value < 0 restores
    the default.  Process-wide; the library reads no environment variable."""
    check(lib().tomatis_set_dev_option(DEV_KEYS[name], int(value)), "set_dev_option")


def get_dev_option(name: str) -> int:
    """The current override of TOMATIS_DEV_<name> (-1: the default)."""
    return int(lib().tomatis_get_dev_option(DEV_KEYS[name]))


class dev_options:
    """Context manager: ``with dev_options(RUN_FRAMES=48, FAST_LOOP=0): ...``
    sets development overrides and restores the values they had on entry
    (nested contexts and earlier set_dev_option calls survive).  The overrides
    are process-wide: set them while no other thread creates plans."""

    def __init__(self, **kw):
        self.kw = kw
        self.saved = {}

    def __enter__(self):
        self.saved = {k: get_dev_option(k) for k in self.kw}
        for k, v in self.kw.items():
            set_dev_option(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self.saved.items():
            set_dev_option(k, v)
        return False
