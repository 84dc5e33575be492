"""ctypes front-end of the CPU ORACLE (test infrastructure only).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import this module.
It loads oracle/build/liboracle.so (built by oracle/Makefile) — the plain-C restatement of
/root/reference/src/fp_handler.c:577-671 (fingerprint) and :247-374 (search).
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "build", "liboracle.so")
NULL_MICRO = -(2**31)


class Tables(C.Structure):
    _fields_ = [
        ("sample_rate", C.c_int),
        ("window", C.c_float * 512),
        ("tw256_re", C.c_float * 256),
        ("tw256_im", C.c_float * 256),
        ("tw512_re", C.c_float * 257),
        ("tw512_im", C.c_float * 257),
        ("mel", (C.c_float * 257) * 40),
        ("dct", (C.c_float * 40) * 2),
    ]


def build(force: bool = False) -> str:
    if force or not os.path.exists(LIB_PATH):
        subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB_PATH


_lib = None
_tables: dict[int, Tables] = {}


def lib():
    global _lib
    if _lib is None:
        build()
        L = C.CDLL(LIB_PATH)
        L.tfo_build_tables.argtypes = [C.c_int, C.POINTER(Tables)]
        L.tfo_frame_count.argtypes = [C.c_size_t]
        L.tfo_frame_count.restype = C.c_size_t
        L.tfo_fingerprint.argtypes = [C.POINTER(Tables), C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]
        L.tfo_fingerprint.restype = C.c_size_t
        L.tfo_fingerprint_f32.argtypes = [C.POINTER(Tables), C.c_void_p, C.c_size_t, C.c_void_p, C.c_void_p, C.c_void_p]
        L.tfo_fingerprint_f32.restype = C.c_size_t
        L.tfo_fingerprint_batch.argtypes = [C.POINTER(Tables), C.c_void_p, C.c_void_p, C.c_int, C.c_void_p, C.c_void_p, C.c_int]
        L.tfo_fingerprint_batch.restype = C.c_size_t
        L.tfo_fingerprint_batch_variant.argtypes = [C.POINTER(Tables), C.c_void_p, C.c_void_p, C.c_int, C.c_void_p,
                                                    C.c_void_p, C.c_int, C.c_int]
        L.tfo_fingerprint_batch_variant.restype = C.c_size_t
        L.tfo_search.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_int64, C.POINTER(C.c_char_p), C.c_int32,
                                 C.c_void_p, C.c_void_p, C.c_int32, C.c_int, C.c_double, C.c_int, C.c_int,
                                 C.POINTER(C.c_int32), C.POINTER(C.c_int32), C.POINTER(C.c_int32)]
        L.tfo_search.restype = C.c_int
        L.tfo_sort_rows.argtypes = [C.c_void_p] * 3 + [C.c_int64] + [C.c_void_p] * 3
        L.tfo_sort_rows.restype = C.c_int64
        L.tfo_search_sorted_batch.argtypes = ([C.c_void_p] * 3 + [C.c_int64, C.c_void_p, C.c_int32] + [C.c_void_p] * 3
                                              + [C.c_int32, C.c_int, C.c_double, C.c_int, C.c_int, C.c_void_p,
                                                 C.c_void_p, C.c_int])
        L.tfo_search_sorted_batch.restype = C.c_int
        L.tfo_search_boxes_batch.argtypes = L.tfo_search_sorted_batch.argtypes + [C.c_int]
        L.tfo_search_boxes_batch.restype = C.c_int
        L.tfo_fmt6.argtypes = [C.c_double]
        L.tfo_fmt6.restype = C.c_int64
        _lib = L
    return _lib


def tables(sample_rate: int = 8000) -> Tables:
    if sample_rate not in _tables:
        t = Tables()
        if lib().tfo_build_tables(sample_rate, C.byref(t)) != 0:
            raise ValueError("bad sample rate")
        _tables[sample_rate] = t
    return _tables[sample_rate]


def table_arrays(sample_rate: int = 8000) -> dict[str, np.ndarray]:
    t = tables(sample_rate)
    return {
        "window": np.ctypeslib.as_array(t.window).copy(),
        "tw256": np.ctypeslib.as_array(t.tw256_re) + 1j * np.ctypeslib.as_array(t.tw256_im).astype(np.float64),
        "mel": np.ctypeslib.as_array(t.mel).reshape(40, 257).copy(),
        "dct": np.ctypeslib.as_array(t.dct).reshape(2, 40).copy(),
    }


def frame_count(n: int) -> int:
    return (n + 255) // 256


def fingerprint(pcm: np.ndarray, sample_rate: int = 8000):
    """-> (coef float32[F,2], db float64[F,2], micro int32[F,2]) for one clip."""
    pcm = np.ascontiguousarray(pcm, dtype=np.int16)
    nf = frame_count(len(pcm))
    coef = np.zeros((nf, 2), np.float32)
    db = np.zeros((nf, 2), np.float64)
    micro = np.zeros((nf, 2), np.int32)
    lib().tfo_fingerprint(C.byref(tables(sample_rate)), pcm.ctypes.data, len(pcm), coef.ctypes.data,
                          db.ctypes.data, micro.ctypes.data)
    return coef, db, micro


def fingerprint_f32(x: np.ndarray, sample_rate: int = 8000):
    """fingerprint() from fp32 hop values (aubio's source output) instead of int16 PCM."""
    x = np.ascontiguousarray(x, dtype=np.float32)
    nf = frame_count(len(x))
    coef = np.zeros((nf, 2), np.float32)
    db = np.zeros((nf, 2), np.float64)
    micro = np.zeros((nf, 2), np.int32)
    lib().tfo_fingerprint_f32(C.byref(tables(sample_rate)), x.ctypes.data, len(x), coef.ctypes.data,
                              db.ctypes.data, micro.ctypes.data)
    return coef, db, micro


def wav_mono_f32(frames: np.ndarray, bits: int, is_float: bool = False) -> np.ndarray:
    """aubio 0.4.5's source output for decoded WAV frames [n, channels] (restated in numpy fp32,
    the restatement tfp_wav_decode_f32 is checked against): per sample (u - 128) / 128 for 8-bit,
    x / 2^(bits-1) for 16/24-bit, fp32(x) * 2^-31 for 32-bit, float data as fp32; then the channels
    summed in fp32 in channel order and divided by the channel count in fp32."""
    f32 = np.float32
    if is_float:
        v = frames.astype(np.float32)
    elif bits == 8:
        v = (frames.astype(np.int32) - 128).astype(f32) / f32(128)
    elif bits == 32:
        v = frames.astype(np.int32).astype(f32) * f32(2.0 ** -31)
    else:
        v = frames.astype(np.int32).astype(f32) / f32(2.0 ** (bits - 1))
    acc = np.zeros(v.shape[0], f32)
    for c in range(v.shape[1]):
        acc = (acc + v[:, c]).astype(f32)
    return (acc / f32(v.shape[1])).astype(f32)


def fingerprint_batch(pcm: np.ndarray, offsets: np.ndarray, sample_rate: int = 8000, nthreads: int = 1,
                      want_db: bool = True, fft_variant: int = 0):
    """fft_variant != 0: another valid fp32 FFT order (tfo_fingerprint_batch_variant)."""
    pcm = np.ascontiguousarray(pcm, dtype=np.int16)
    offsets = np.ascontiguousarray(offsets, dtype=np.int64)
    nclips = len(offsets) - 1
    total = int(sum(frame_count(int(offsets[i + 1] - offsets[i])) for i in range(nclips)))
    micro = np.zeros((total, 2), np.int32)
    db = np.zeros((total, 2), np.float64) if want_db else None
    lib().tfo_fingerprint_batch_variant(C.byref(tables(sample_rate)), pcm.ctypes.data, offsets.ctypes.data, nclips,
                                        micro.ctypes.data, db.ctypes.data if db is not None else None, nthreads,
                                        fft_variant)
    return micro, db


def search(m1, m2, row_clip, uuids, q1, q2, coefs=1, tolerance=0.001, low=-1, high=-1):
    """fp_search_fingerprint_info semantics -> (found, winner_index, match_count, frame_count)."""
    m1 = np.ascontiguousarray(m1, np.int32)
    m2 = np.ascontiguousarray(m2, np.int32)
    row_clip = np.ascontiguousarray(row_clip, np.int32)
    q1 = np.ascontiguousarray(q1, np.float64)
    q2 = np.ascontiguousarray(q2, np.float64)
    arr = (C.c_char_p * max(1, len(uuids)))(*[u.encode() for u in uuids])
    w, mc, fc = C.c_int32(), C.c_int32(), C.c_int32()
    found = lib().tfo_search(m1.ctypes.data, m2.ctypes.data, row_clip.ctypes.data, len(m1), arr, len(uuids),
                             q1.ctypes.data, q2.ctypes.data, len(q1), coefs, float(tolerance), int(low), int(high),
                             C.byref(w), C.byref(mc), C.byref(fc))
    return bool(found), w.value, mc.value, fc.value


class SortedIndex:
    """The audio_fingerprint rows ordered by max1 (idx_audio_fingerprint_max1) for searches over
    large tables; tiekey[clip] = rank of the clip's uuid (greatest wins a tie)."""

    def __init__(self, m1, m2, row_clip, tiekey):
        m1 = np.ascontiguousarray(m1, np.int32)
        m2 = np.ascontiguousarray(m2, np.int32)
        row_clip = np.ascontiguousarray(row_clip, np.int32)
        n = len(m1)
        self.m1 = np.empty(n, np.int32)
        self.m2 = np.empty(n, np.int32)
        self.clip = np.empty(n, np.int32)
        if lib().tfo_sort_rows(m1.ctypes.data, m2.ctypes.data, row_clip.ctypes.data, n, self.m1.ctypes.data,
                               self.m2.ctypes.data, self.clip.ctypes.data) != n:
            raise MemoryError("tfo_sort_rows")
        self.tiekey = np.ascontiguousarray(tiekey, np.int32)

    def search_batch(self, q1, q2, qoff, coefs=1, tolerance=0.001, low=-1, high=-1, nthreads=8, method="scan",
                     mode=0):
        """-> (winner clip int32[nq] (-1 = NOTFOUND), match_count int32[nq]). method "scan": one row
        scan per distinct frame clause (tfo_search_sorted_batch); "boxes": per distinct max1 box, max2
        runs or per-clip merges (tfo_search_boxes_batch; mode 1/2 forces one form), for wide
        coefs = 2 windows at configs[2] size."""
        q1 = np.ascontiguousarray(q1, np.float64)
        q2 = np.ascontiguousarray(q2, np.float64)
        qoff = np.ascontiguousarray(qoff, np.int64)
        nq = len(qoff) - 1
        w = np.zeros(nq, np.int32)
        mc = np.zeros(nq, np.int32)
        args = (self.m1.ctypes.data, self.m2.ctypes.data, self.clip.ctypes.data, len(self.m1), self.tiekey.ctypes.data,
                len(self.tiekey), q1.ctypes.data, q2.ctypes.data, qoff.ctypes.data, nq, coefs, float(tolerance), int(low),
                int(high), w.ctypes.data, mc.ctypes.data, int(nthreads))
        if method == "boxes":
            if lib().tfo_search_boxes_batch(*args, int(mode)) != 0:
                raise MemoryError("tfo_search_boxes_batch")
        else:
            lib().tfo_search_sorted_batch(*args)
        return w, mc


def fmt6(x: float) -> int:
    return int(lib().tfo_fmt6(float(x)))
