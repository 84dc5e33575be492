"""The C-ABI library loads, exports every symbol include/tiresias_fp.h declares, and its
host-only entry points behave (no GPU compute here)."""
import ctypes as C

import numpy as np


def test_exports_every_header_symbol(tfp_lib):
    syms = tfp_lib.header_symbols()
    assert len(syms) >= 25
    L = C.CDLL(tfp_lib.LIB_PATH)
    missing = [s for s in syms if not hasattr(L, s)]
    assert not missing, missing


def test_abi_version_and_frame_count(tfp_lib):
    L = tfp_lib.lib()
    assert L.tfp_abi_version() == 1
    for n, f in [(0, 0), (1, 1), (255, 1), (256, 1), (257, 2), (80000, 313), (240000, 938), (40000, 157),
                 (24000, 94), (-5, 0)]:
        assert L.tfp_frame_count(n) == f


def test_synth_deterministic(tfp_lib):
    a = tfp_lib.synth_pcm(0x7153A1, [0, 1, 2], 5000)
    b = tfp_lib.synth_pcm(0x7153A1, [0, 1, 2], 5000)
    assert np.array_equal(a, b)
    assert a.dtype == np.int16 and a.shape == (3, 5000)
    assert not np.array_equal(a[0], a[1])
    # offsets: excerpt of clip 1 starting at sample 512
    c = tfp_lib.synth_pcm(0x7153A1, [1], 1000, offsets=[512])
    assert np.array_equal(c[0], a[1, 512:1512])
    peak = np.abs(a.astype(np.int32)).max()
    assert 4000 < peak < 32768


def test_engine_create_without_gpu_fails_cleanly(tfp_lib):
    if tfp_lib.device_count() > 0:
        return
    import pytest
    with pytest.raises(tfp_lib.TfpError):
        tfp_lib.Engine(0)
