"""Audio ingest (tfp_wav_decode / tfp_wav_read, include/tiresias_fp.h): the aubio_source step in
front of create_audio_fingerprints (/root/reference/src/fp_handler.c:37, :604, :633). Host-only
calls into the C-ABI library, so these run without a GPU.

aubio's value for a w-bit integer sample x is x / 2^(w-1) (8-bit: (u - 128) / 128). The engine
computes s / 32768 from int16 s, so 16-bit data must come back as stored and 8-bit data as
(u - 128) << 8. Audio whose aubio value lies between int16 steps must be refused."""
import struct

import numpy as np
import pytest

from tiresias_amd import TfpError
from tiresias_amd._lib import lib
from tiresias_amd.engine import decode_wav, read_wav
from tiresias_amd.fp_handler import write_wav_mono16

TFP_E_CAPACITY, TFP_E_FORMAT, TFP_E_NOENT = -5, -8, -4


def chunk(cid: bytes, body: bytes) -> bytes:
    return cid + struct.pack("<I", len(body)) + body + (b"\0" if len(body) & 1 else b"")


def fmt_pcm(channels=1, rate=8000, bits=16, tag=1):
    align = channels * bits // 8
    return chunk(b"fmt ", struct.pack("<HHIIHH", tag, channels, rate, rate * align, align, bits))


def fmt_extensible(sub_tag=1, channels=1, rate=8000, bits=16):
    align = channels * bits // 8
    guid = struct.pack("<H", sub_tag) + b"\x00\x00\x00\x00\x10\x00\x80\x00\x00\xaa\x00\x38\x9b\x71"
    body = struct.pack("<HHIIHHHHI", 0xFFFE, channels, rate, rate * align, align, bits, 22, bits, 4) + guid
    return chunk(b"fmt ", body)


def riff(*chunks: bytes) -> bytes:
    body = b"WAVE" + b"".join(chunks)
    return b"RIFF" + struct.pack("<I", len(body)) + body


def test_16bit_mono_matches_python_wave(tmp_path):
    rng = np.random.default_rng(5)
    for n, sr in ((0, 8000), (1, 8000), (80000, 8000), (12345, 16000), (4411, 44100)):
        pcm = rng.integers(-32768, 32768, n, dtype=np.int16)
        path = str(tmp_path / f"c{n}.wav")
        write_wav_mono16(path, pcm, sr)
        got, got_sr = read_wav(path)
        assert got_sr == sr and got.dtype == np.int16
        np.testing.assert_array_equal(got, pcm)
        got2, _ = decode_wav(open(path, "rb").read())
        np.testing.assert_array_equal(got2, pcm)


def test_asterisk_format_wav_header():
    """format_wav's header (16-byte fmt, PCM mono 16-bit 8 kHz), as the dialplan recording
    (application_handler.c:155) writes it."""
    pcm = np.arange(-600, 600, 3, dtype=np.int16)
    got, sr = decode_wav(riff(fmt_pcm(), chunk(b"data", pcm.tobytes())))
    assert sr == 8000
    np.testing.assert_array_equal(got, pcm)


def test_8bit_maps_exactly_onto_int16():
    u = np.arange(256, dtype=np.uint8)
    got, _ = decode_wav(riff(fmt_pcm(bits=8), chunk(b"data", u.tobytes())))
    np.testing.assert_array_equal(got.astype(np.int32), (u.astype(np.int32) - 128) * 256)
    # aubio's fp32 value (u - 128) / 128 equals the engine's s / 32768
    np.testing.assert_array_equal(got.astype(np.float32) / np.float32(32768),
                                  (u.astype(np.float32) - 128) / np.float32(128))


def test_chunks_skipped_and_padded():
    pcm = np.array([1, -2, 3, 32767, -32768], np.int16)
    data = riff(chunk(b"LIST", b"INFOabc"), fmt_pcm(), chunk(b"fact", b"\x05\0\0\0"), chunk(b"data", pcm.tobytes()),
                chunk(b"junk", b"zz"))
    got, _ = decode_wav(data)
    np.testing.assert_array_equal(got, pcm)


def test_extensible_pcm_accepted_float_refused():
    pcm = np.array([7, -7, 100], np.int16)
    got, _ = decode_wav(riff(fmt_extensible(), chunk(b"data", pcm.tobytes())))
    np.testing.assert_array_equal(got, pcm)
    with pytest.raises(TfpError) as e:
        decode_wav(riff(fmt_extensible(sub_tag=3, bits=32), chunk(b"data", b"\0" * 8)))
    assert e.value.code == TFP_E_FORMAT


@pytest.mark.parametrize("fmt", [fmt_pcm(channels=2), fmt_pcm(bits=24), fmt_pcm(bits=32), fmt_pcm(tag=3, bits=32),
                                 fmt_pcm(tag=7, bits=8)])
def test_inexact_audio_refused(fmt):
    with pytest.raises(TfpError) as e:
        decode_wav(riff(fmt, chunk(b"data", b"\0" * 12)))
    assert e.value.code == TFP_E_FORMAT
    assert lib().tfp_engine_last_error(None)  # the reason is reported


def test_unpatched_and_truncated_data_sizes():
    pcm = np.arange(10, dtype=np.int16)
    body = pcm.tobytes()
    for size in (0, 0xFFFFFFFF, 1000):
        raw = riff(fmt_pcm()) + b"data" + struct.pack("<I", size) + body
        got, _ = decode_wav(raw)
        np.testing.assert_array_equal(got, pcm)
    got, _ = decode_wav(riff(fmt_pcm()) + b"data" + struct.pack("<I", 20) + body[:7])  # half a sample dropped
    np.testing.assert_array_equal(got, pcm[:3])


@pytest.mark.parametrize("raw", [b"", b"RIFF", b"RIFX\0\0\0\0WAVE", b"RIFF\0\0\0\0AVI ",
                                 riff(chunk(b"data", b"\0\0")), riff(fmt_pcm()), riff(chunk(b"fmt ", b"\1\0"))])
def test_malformed_refused(raw):
    with pytest.raises(TfpError) as e:
        decode_wav(raw)
    assert e.value.code == TFP_E_FORMAT


def test_capacity_and_missing_file(tmp_path):
    import ctypes as C
    raw = riff(fmt_pcm(), chunk(b"data", np.arange(8, dtype=np.int16).tobytes()))
    out = np.zeros(4, np.int16)
    n, sr = C.c_int64(), C.c_int32()
    rc = lib().tfp_wav_decode(raw, len(raw), out.ctypes.data, 4, C.byref(n), C.byref(sr))
    assert rc == TFP_E_CAPACITY and n.value == 8
    with pytest.raises(TfpError) as e:
        read_wav(str(tmp_path / "absent.wav"))
    assert e.value.code == TFP_E_NOENT


# ---- fp32 form (tfp_wav_decode_f32): every encoding, channels averaged as aubio does ---------
def _frames(rng, n, ch, bits, is_float=False):
    if is_float:
        return (rng.standard_normal((n, ch)) * 0.3).astype(np.float64 if bits == 64 else np.float32)
    if bits == 8:
        return rng.integers(0, 256, (n, ch)).astype(np.uint8)
    lo, hi = -(1 << (bits - 1)), 1 << (bits - 1)
    x = rng.integers(lo, hi, (n, ch), dtype=np.int64)
    x[:3] = [[lo] * ch, [hi - 1] * ch, [0] * ch][:min(3, n)]  # extremes
    return x


def _data_bytes(fr, bits, is_float):
    if is_float:
        return fr.astype("<f8" if bits == 64 else "<f4").tobytes()
    if bits == 8:
        return fr.astype(np.uint8).tobytes()
    if bits == 24:
        u = fr.astype(np.int64).reshape(-1) & 0xFFFFFF
        return np.stack([u & 0xFF, (u >> 8) & 0xFF, (u >> 16) & 0xFF], 1).astype(np.uint8).tobytes()
    return fr.astype("<i2" if bits == 16 else "<i4").tobytes()


@pytest.mark.parametrize("ch,bits,is_float", [(2, 16, False), (3, 16, False), (6, 16, False), (2, 8, False),
                                              (1, 24, False), (2, 24, False), (1, 32, False), (2, 32, False),
                                              (1, 32, True), (2, 32, True), (2, 64, True), (1, 16, False)])
def test_f32_decode_equals_aubio_restatement(oracle, ch, bits, is_float):
    """Parity of the fp32 ingest with oracle_py.wav_mono_f32 (the numpy restatement of aubio
    0.4.5's sndfile/wavread conversion and channel mean), bit for bit."""
    from tiresias_amd.engine import decode_wav_f32
    rng = np.random.default_rng(ch * 100 + bits)
    fr = _frames(rng, 5000, ch, bits, is_float)
    raw = riff(fmt_pcm(ch, 16000, bits, 3 if is_float else 1), chunk(b"data", _data_bytes(fr, bits, is_float)))
    x, sr = decode_wav_f32(raw)
    assert sr == 16000 and x.dtype == np.float32 and len(x) == 5000
    want = oracle.wav_mono_f32(fr, bits, is_float)
    np.testing.assert_array_equal(x.view(np.uint32), want.view(np.uint32))


def test_f32_decode_of_int16_mono_is_pcm_over_32768():
    """On the int16 path's inputs the fp32 form is exactly s / 32768 (so both entry points give
    the same fingerprints); 8-bit likewise ((u - 128) << 8) / 32768."""
    from tiresias_amd.engine import decode_wav_f32
    pcm = np.arange(-32768, 32768, 7, dtype=np.int16)
    x, _ = decode_wav_f32(riff(fmt_pcm(), chunk(b"data", pcm.tobytes())))
    np.testing.assert_array_equal(x, pcm.astype(np.float32) / np.float32(32768))
    u = np.arange(256, dtype=np.uint8)
    x8, _ = decode_wav_f32(riff(fmt_pcm(bits=8), chunk(b"data", u.tobytes())))
    p8, _ = decode_wav(riff(fmt_pcm(bits=8), chunk(b"data", u.tobytes())))
    np.testing.assert_array_equal(x8, p8.astype(np.float32) / np.float32(32768))


def test_f32_decode_extensible_and_errors(tmp_path):
    from tiresias_amd.engine import decode_wav_f32, read_wav_f32
    v = np.array([0.5, -0.25, 1.0, 0.125], np.float32)
    x, _ = decode_wav_f32(riff(fmt_extensible(3, 1, 8000, 32), chunk(b"data", v.tobytes())))
    np.testing.assert_array_equal(x, v)
    with pytest.raises(TfpError) as e:  # 12-bit PCM: not a supported width
        decode_wav_f32(riff(fmt_pcm(1, 8000, 12), chunk(b"data", b"\0" * 8)))
    assert e.value.code == TFP_E_FORMAT
    with pytest.raises(TfpError) as e:  # A-law
        decode_wav_f32(riff(fmt_pcm(1, 8000, 8, tag=6), chunk(b"data", b"\0" * 8)))
    assert e.value.code == TFP_E_FORMAT
    path = tmp_path / "st.wav"
    st = np.array([[100, -100], [32767, 32767], [-32768, 1]], np.int16)
    path.write_bytes(riff(fmt_pcm(2), chunk(b"data", st.tobytes())))
    x, sr = read_wav_f32(str(path))
    assert sr == 8000
    np.testing.assert_array_equal(x, np.array([0.0, 32767 / 32768, -32767 / 65536], np.float32))
    with pytest.raises(TfpError) as e:
        read_wav_f32(str(tmp_path / "missing.wav"))
    assert e.value.code == TFP_E_NOENT
