"""tiresias_amd — MI355X-native fingerprint engine for asterisk-tiresias (Python side).

The compute lives in lib/libtiresias_fp.so (HIP, gfx950) behind include/tiresias_fp.h;
this package is its ctypes binding plus a mirror of the reference's fp_handler interface.
"""
from ._lib import LIB_PATH, NULL_MICRO, TfpError, header_symbols, lib  # noqa: F401
from .engine import (FRAME_DTYPE, Engine, Group, GroupStream, Plan, Stream, device_count, frame_count,  # noqa: F401
                     params, synth_pcm)
from .fp_handler import FpHandler  # noqa: F401
