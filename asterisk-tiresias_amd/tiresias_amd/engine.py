"""Pythonic wrapper of the C-ABI engine (numpy in/out)."""
from __future__ import annotations

import ctypes as C
import weakref

import numpy as np

from ._lib import Frame, Result, SearchParams, SynthSpec, TfpError, check, lib

FRAME_DTYPE = np.dtype([("frame_idx", "<i4"), ("m1", "<i4"), ("m2", "<i4"), ("reserved", "<i4"),
                        ("q1", "<f8"), ("q2", "<f8")])
assert FRAME_DTYPE.itemsize == C.sizeof(Frame) == 32


def device_count() -> int:
    n = C.c_int32()
    rc = lib().tfp_device_count(C.byref(n))
    return n.value if rc == 0 else 0


def frame_count(nsamples: int) -> int:
    return int(lib().tfp_frame_count(int(nsamples)))


def params(coefs=1, tolerance=-1.0, freq_ignore_low=-1, freq_ignore_high=-1) -> SearchParams:
    return SearchParams(int(coefs), int(freq_ignore_low), int(freq_ignore_high), 0, float(tolerance))


def _wav(call, dtype=np.int16) -> tuple[np.ndarray, int]:
    n, sr = C.c_int64(), C.c_int32()
    check(call(None, 0, C.byref(n), C.byref(sr)))
    pcm = np.empty(n.value, dtype)
    check(call(pcm.ctypes.data, n.value, C.byref(n), C.byref(sr)))
    return pcm, sr.value


def decode_wav(data: bytes) -> tuple[np.ndarray, int]:
    """tfp_wav_decode: RIFF/WAVE bytes -> (mono int16 PCM, native rate), aubio_source semantics
    (fp_handler.c:37, :604, :633). TfpError(TFP_E_FORMAT) for audio the engine cannot take exactly."""
    buf = C.create_string_buffer(bytes(data), len(data))
    return _wav(lambda pcm, cap, n, sr: lib().tfp_wav_decode(buf, len(data), pcm, cap, n, sr))


def read_wav(path: str) -> tuple[np.ndarray, int]:
    """tfp_wav_read: decode_wav of a file."""
    p = path.encode()
    return _wav(lambda pcm, cap, n, sr: lib().tfp_wav_read(p, pcm, cap, n, sr))


def decode_wav_f32(data: bytes) -> tuple[np.ndarray, int]:
    """tfp_wav_decode_f32: RIFF/WAVE bytes -> (fp32 mono hop values as aubio_source computes them,
    native rate), for every PCM width / float format and channel count."""
    buf = C.create_string_buffer(bytes(data), len(data))
    return _wav(lambda x, cap, n, sr: lib().tfp_wav_decode_f32(buf, len(data), x, cap, n, sr), np.float32)


def read_wav_f32(path: str) -> tuple[np.ndarray, int]:
    """tfp_wav_read_f32: decode_wav_f32 of a file."""
    p = path.encode()
    return _wav(lambda x, cap, n, sr: lib().tfp_wav_read_f32(p, x, cap, n, sr), np.float32)


def synth_specs(seed: int, clips, offsets=None):
    clips = list(clips)
    offsets = [0] * len(clips) if offsets is None else list(offsets)
    arr = (SynthSpec * max(1, len(clips)))()
    for i, (c, o) in enumerate(zip(clips, offsets)):
        arr[i] = SynthSpec(seed & (2**64 - 1), int(c), int(o))
    return arr


def synth_pcm(seed: int, clips, samples_per_clip: int, offsets=None) -> np.ndarray:
    """Deterministic synthetic PCM (host side of tfp_synth_pcm) -> int16[nclips, samples]."""
    clips = list(clips)
    out = np.zeros((len(clips), samples_per_clip), np.int16)
    specs = synth_specs(seed, clips, offsets)
    check(lib().tfp_synth_pcm(specs, len(clips), samples_per_clip, out.ctypes.data))
    return out


class Engine:
    """One engine per GPU (tfp_engine)."""

    def __init__(self, device: int = 0):
        self._h = C.c_void_p()
        rc = lib().tfp_engine_create(int(device), C.byref(self._h))
        if rc != 0:
            raise TfpError(rc, f"cannot create engine on device {device}")
        self.device = device
        self._streams = weakref.WeakSet()  # live Streams: destroyed before the engine (tiresias_fp.h)

    def close(self):
        if self._h:
            for st in list(self._streams):
                st.close()
            lib().tfp_engine_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    @property
    def handle(self):
        return self._h

    def _chk(self, rc):
        return check(rc, self._h)

    # ---- fingerprinting -----------------------------------------------------------
    def fingerprint(self, pcm: np.ndarray, sample_rate: int = 8000) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, np.int16)
        n = frame_count(len(pcm))
        out = np.zeros(n, FRAME_DTYPE)
        got = C.c_int64()
        self._chk(lib().tfp_fingerprint_pcm(self._h, pcm.ctypes.data, len(pcm), sample_rate, out.ctypes.data, n,
                                            C.byref(got)))
        return out

    def fingerprint_batch(self, pcm: np.ndarray, offsets, sample_rate: int = 8000) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, np.int16)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nclips = len(offsets) - 1
        n = sum(frame_count(int(offsets[i + 1] - offsets[i])) for i in range(nclips))
        out = np.zeros(max(n, 1), FRAME_DTYPE)
        got = C.c_int64()
        self._chk(lib().tfp_fingerprint_batch(self._h, pcm.ctypes.data, offsets.ctypes.data, nclips, sample_rate,
                                              out.ctypes.data, n, C.byref(got)))
        return out[:n]

    def fingerprint_f32_batch(self, x: np.ndarray, offsets, sample_rate: int = 8000) -> np.ndarray:
        """tfp_fingerprint_f32_batch: fingerprint_batch over fp32 hop values (decode_wav_f32)."""
        x = np.ascontiguousarray(x, np.float32)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nclips = len(offsets) - 1
        n = sum(frame_count(int(offsets[i + 1] - offsets[i])) for i in range(nclips))
        out = np.zeros(max(n, 1), FRAME_DTYPE)
        got = C.c_int64()
        self._chk(lib().tfp_fingerprint_f32_batch(self._h, x.ctypes.data, offsets.ctypes.data, nclips, sample_rate,
                                                  out.ctypes.data, n, C.byref(got)))
        return out[:n]

    # ---- index ----------------------------------------------------------------------
    def index_add(self, uuid: str, m1, m2) -> int:
        m1 = np.ascontiguousarray(m1, np.int32)
        m2 = np.ascontiguousarray(m2, np.int32)
        cid = C.c_int32()
        self._chk(lib().tfp_index_add(self._h, uuid.encode(), m1.ctypes.data, m2.ctypes.data, len(m1), C.byref(cid)))
        return cid.value

    def index_add_batch(self, uuids, frame_offsets, m1, m2):
        frame_offsets = np.ascontiguousarray(frame_offsets, np.int64)
        m1 = np.ascontiguousarray(m1, np.int32)
        m2 = np.ascontiguousarray(m2, np.int32)
        arr = (C.c_char_p * max(1, len(uuids)))(*[u.encode() for u in uuids])
        self._chk(lib().tfp_index_add_batch(self._h, len(uuids), arr, frame_offsets.ctypes.data, m1.ctypes.data,
                                            m2.ctypes.data))

    def index_rows(self, uuid: str):
        """Stored (m1, m2) micro-unit rows of one clip, frame order."""
        n = C.c_int64()
        rc = lib().tfp_index_rows(self._h, uuid.encode(), None, None, 0, C.byref(n))
        if rc not in (0, -5):
            self._chk(rc)
        m1 = np.zeros(max(n.value, 1), np.int32)
        m2 = np.zeros(max(n.value, 1), np.int32)
        self._chk(lib().tfp_index_rows(self._h, uuid.encode(), m1.ctypes.data, m2.ctypes.data, n.value, C.byref(n)))
        return m1[:n.value], m2[:n.value]

    def index_remove(self, uuid: str):
        self._chk(lib().tfp_index_remove(self._h, uuid.encode()))

    def index_clear(self):
        self._chk(lib().tfp_index_clear(self._h))

    def index_stats(self):
        r, c = C.c_int64(), C.c_int32()
        self._chk(lib().tfp_index_stats(self._h, C.byref(r), C.byref(c)))
        return r.value, c.value

    def index_commit(self):
        self._chk(lib().tfp_index_commit(self._h))

    def index_build_stats(self):
        """(full builds, incremental merges) of the sorted index so far."""
        f, m = C.c_int64(), C.c_int64()
        self._chk(lib().tfp_index_build_stats(self._h, C.byref(f), C.byref(m)))
        return f.value, m.value

    def index_delta_stats(self):
        """(delta updates so far, clips in the index delta now)."""
        u, c = C.c_int64(), C.c_int32()
        self._chk(lib().tfp_index_delta_stats(self._h, C.byref(u), C.byref(c)))
        return u.value, c.value

    def sweep_stats(self) -> dict:
        """The coefs = 2 sweep's sort path per batch (tfp_sweep_stats): bin sort, library sort,
        redone speculative passes, crowd bins copied."""
        v = [C.c_int64() for _ in range(4)]
        self._chk(lib().tfp_sweep_stats(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("bins", "library", "redone", "crowd"), [x.value for x in v]))

    def index_cache_stats(self) -> dict:
        """The coefs = 2 clip-set caches (tfp_index_cache_stats): builds, cached hits, builds from the
        clip order, the clip order's full builds and merges, the index delta's caches and sweeps."""
        v = [C.c_int64() for _ in range(7)]
        self._chk(lib().tfp_index_cache_stats(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("builds", "hits", "from_order", "order_builds", "order_merges", "delta_builds", "delta_sweeps"),
                        [x.value for x in v]))

    def set_tiebreak(self, keys):
        keys = np.ascontiguousarray(keys, np.int32)
        self._chk(lib().tfp_index_set_tiebreak(self._h, keys.ctypes.data, len(keys)))

    def update_tiebreak(self, first_clip_id: int, keys):
        """tfp_index_update_tiebreak: the override's keys of clip ids first_clip_id.. only."""
        keys = np.ascontiguousarray(keys, np.int32)
        self._chk(lib().tfp_index_update_tiebreak(self._h, int(first_clip_id), keys.ctypes.data, len(keys)))

    def uuid_of_key(self, key: int) -> str:
        buf = C.create_string_buffer(64)
        self._chk(lib().tfp_index_uuid_of_key(self._h, int(key), buf, 64))
        return buf.value.decode()

    # ---- search ---------------------------------------------------------------------
    @staticmethod
    def _results(res, n):
        return [None if not r.found else {"audio_uuid": r.uuid.decode(), "match_count": r.match_count,
                                          "frame_count": r.frame_count, "clip_id": r.clip_id}
                for r in res[:n]], [r.frame_count for r in res[:n]]

    def search_batch(self, frames: np.ndarray, qoffsets, p: SearchParams):
        frames = np.ascontiguousarray(frames, FRAME_DTYPE)
        qoffsets = np.ascontiguousarray(qoffsets, np.int64)
        nq = len(qoffsets) - 1
        res = (Result * max(1, nq))()
        self._chk(lib().tfp_search_batch(self._h, frames.ctypes.data, qoffsets.ctypes.data, nq, C.byref(p), res))
        return self._results(res, nq)

    def search(self, frames: np.ndarray, p: SearchParams):
        r, fc = self.search_batch(frames, [0, len(frames)], p)
        return r[0], fc[0]

    def search_pcm_batch(self, pcm: np.ndarray, offsets, p: SearchParams, sample_rate: int = 8000):
        pcm = np.ascontiguousarray(pcm, np.int16)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nq = len(offsets) - 1
        res = (Result * max(1, nq))()
        self._chk(lib().tfp_search_pcm_batch(self._h, pcm.ctypes.data, offsets.ctypes.data, nq, sample_rate,
                                             C.byref(p), res))
        return self._results(res, nq)

    def search_f32_batch(self, x: np.ndarray, offsets, p: SearchParams, sample_rate: int = 8000):
        """tfp_search_f32_batch: search_pcm_batch over fp32 hop values."""
        x = np.ascontiguousarray(x, np.float32)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nq = len(offsets) - 1
        res = (Result * max(1, nq))()
        self._chk(lib().tfp_search_f32_batch(self._h, x.ctypes.data, offsets.ctypes.data, nq, sample_rate,
                                             C.byref(p), res))
        return self._results(res, nq)

    # ---- device-resident paths (pointers are raw device addresses, e.g. tensor.data_ptr())
    def plan(self, offsets, sample_rate: int = 8000) -> "Plan":
        return Plan(self, offsets, sample_rate)

    def fingerprint_device(self, plan: "Plan", d_pcm: int, d_micro: int, d_db: int = 0, stream: int = 0):
        self._chk(lib().tfp_fingerprint_device(self._h, plan.handle, C.c_void_p(d_pcm), C.c_void_p(d_micro),
                                               C.c_void_p(d_db or None), C.c_void_p(stream or None)))

    def index_add_device(self, uuids, frame_offsets, d_micro: int, stream: int = 0):
        frame_offsets = np.ascontiguousarray(frame_offsets, np.int64)
        arr = (C.c_char_p * max(1, len(uuids)))(*[u.encode() for u in uuids])
        self._chk(lib().tfp_index_add_device(self._h, len(uuids), arr, frame_offsets.ctypes.data,
                                             C.c_void_p(d_micro), C.c_void_p(stream or None)))

    def search_device(self, plan: "Plan", d_pcm: int, p: SearchParams, d_keys: int, stream: int = 0):
        self._chk(lib().tfp_search_device(self._h, plan.handle, C.c_void_p(d_pcm), C.byref(p), C.c_void_p(d_keys),
                                          C.c_void_p(stream or None)))

    def search_q_device(self, d_q: int, qoffsets, p: SearchParams, d_keys: int, stream: int = 0):
        """tfp_search_q_device: search from device-resident frame values (2 doubles per frame)."""
        qoffsets = np.ascontiguousarray(qoffsets, np.int64)
        self._chk(lib().tfp_search_q_device(self._h, C.c_void_p(d_q), qoffsets.ctypes.data, len(qoffsets) - 1,
                                            C.byref(p), C.c_void_p(d_keys), C.c_void_p(stream or None)))

    def synth_device(self, seed: int, clips, samples_per_clip: int, d_out: int, offsets=None, stream: int = 0):
        clips = list(clips)
        specs = synth_specs(seed, clips, offsets)
        self._chk(lib().tfp_synth_pcm_device(self._h, specs, len(clips), samples_per_clip, C.c_void_p(d_out),
                                             C.c_void_p(stream or None)))

    def synchronize(self, stream: int = 0):
        self._chk(lib().tfp_synchronize(self._h, C.c_void_p(stream or None)))


class Stream:
    """Live channels (tfp_stream): rolling window fingerprint + match per tick."""

    def __init__(self, eng: Engine, nchannels: int, window_samples: int, sample_rate: int = 8000):
        self._eng = eng
        self._h = C.c_void_p()
        eng._chk(lib().tfp_stream_create(eng.handle, int(nchannels), int(sample_rate), int(window_samples),
                                         C.byref(self._h)))
        self.nchannels = nchannels
        self._res = (Result * nchannels)()
        eng._streams.add(self)

    def reset(self, channel: int = -1):
        self._eng._chk(lib().tfp_stream_reset(self._h, int(channel)))

    def push(self, pcm: np.ndarray, p: SearchParams = None):
        """pcm int16[nchannels, tick] -> list of per-channel results (None = NOTFOUND / not full)."""
        pcm = np.ascontiguousarray(pcm, np.int16)
        assert pcm.shape[0] == self.nchannels
        self._eng._chk(lib().tfp_stream_push(self._h, pcm.ctypes.data, pcm.shape[1],
                                             C.byref(p) if p is not None else None, self._res if p is not None else None))
        if p is None:
            return None
        return [None if not r.found else {"audio_uuid": r.uuid.decode(), "match_count": r.match_count,
                                          "frame_count": r.frame_count} for r in self._res]

    def close(self):
        # tfp_stream_destroy uses the engine: a stream outliving its engine's close() was already
        # destroyed by it, so there is nothing left to free here
        if self._h and self._eng._h:
            lib().tfp_stream_destroy(self._h)
        self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class Plan:
    def __init__(self, eng: Engine, offsets, sample_rate: int = 8000):
        offsets = np.ascontiguousarray(offsets, np.int64)
        self._h = C.c_void_p()
        eng._chk(lib().tfp_plan_create(eng.handle, offsets.ctypes.data, len(offsets) - 1, sample_rate,
                                       C.byref(self._h)))
        self.nframes = int(lib().tfp_plan_frames(self._h))
        self.offsets = offsets

    @property
    def handle(self):
        return self._h

    def __del__(self):
        if self._h:
            lib().tfp_plan_destroy(self._h)
            self._h = C.c_void_p()


class Group:
    """tfp_group: one engine per listed device (a device may repeat), the enrolled clips sharded
    over them, searches combined on the host (tiresias_fp.h, device groups)."""

    def __init__(self, devices):
        devs = (C.c_int32 * len(devices))(*[int(d) for d in devices])
        self._h = C.c_void_p()
        rc = lib().tfp_group_create(devs, len(devices), C.byref(self._h))
        if rc != 0:
            raise TfpError(rc, f"cannot create a group on devices {list(devices)}")
        self.devices = list(devices)
        self._streams = weakref.WeakSet()

    def close(self):
        if self._h:
            for st in list(self._streams):
                st.close()
            lib().tfp_group_destroy(self._h)
            self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def _chk(self, rc):
        if rc != 0:
            raise TfpError(rc, lib().tfp_group_last_error(self._h).decode())
        return rc

    def size(self) -> int:
        return int(lib().tfp_group_size(self._h))

    def tiebreak_stats(self) -> dict:
        """tfp_group_tiebreak_stats: key respaces, new-clip-only pushes, shard delta updates that
        re-sent every main column's key."""
        v = [C.c_int64() for _ in range(3)]
        check(lib().tfp_group_tiebreak_stats(self._h, *[C.byref(x) for x in v]))
        return dict(zip(("respaces", "partial_pushes", "shard_full_key_updates"), [x.value for x in v]))

    def peer_stats(self) -> dict:
        """Peer access among the group's distinct devices (tfp_group_peer_stats): ordered pairs,
        how many may access each other, for how many it is enabled."""
        a, b, c = C.c_int32(), C.c_int32(), C.c_int32()
        check(lib().tfp_group_peer_stats(self._h, C.byref(a), C.byref(b), C.byref(c)))
        return {"pairs": a.value, "can_access": b.value, "enabled": c.value}

    def engine_stats(self):
        """[(rows, clips)] of every shard's engine."""
        out = []
        for s in range(self.size()):
            r, c = C.c_int64(), C.c_int32()
            check(lib().tfp_index_stats(lib().tfp_group_engine(self._h, s), C.byref(r), C.byref(c)))
            out.append((r.value, c.value))
        return out

    def fingerprint_batch(self, pcm, offsets, sample_rate: int = 8000) -> np.ndarray:
        pcm = np.ascontiguousarray(pcm, np.int16)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nclips = len(offsets) - 1
        n = sum(frame_count(int(offsets[i + 1] - offsets[i])) for i in range(nclips))
        out = np.zeros(max(n, 1), FRAME_DTYPE)
        got = C.c_int64()
        self._chk(lib().tfp_group_fingerprint_batch(self._h, pcm.ctypes.data, offsets.ctypes.data, nclips, sample_rate,
                                                    out.ctypes.data, n, C.byref(got)))
        return out[:n]

    def index_add(self, uuid: str, m1, m2):
        m1 = np.ascontiguousarray(m1, np.int32)
        m2 = np.ascontiguousarray(m2, np.int32)
        self._chk(lib().tfp_group_index_add(self._h, uuid.encode(), m1.ctypes.data, m2.ctypes.data, len(m1)))

    def index_add_batch(self, uuids, frame_offsets, m1, m2):
        frame_offsets = np.ascontiguousarray(frame_offsets, np.int64)
        m1 = np.ascontiguousarray(m1, np.int32)
        m2 = np.ascontiguousarray(m2, np.int32)
        arr = (C.c_char_p * max(1, len(uuids)))(*[u.encode() for u in uuids])
        self._chk(lib().tfp_group_index_add_batch(self._h, len(uuids), arr, frame_offsets.ctypes.data, m1.ctypes.data,
                                                  m2.ctypes.data))

    def index_remove(self, uuid: str):
        self._chk(lib().tfp_group_index_remove(self._h, uuid.encode()))

    def index_clear(self):
        self._chk(lib().tfp_group_index_clear(self._h))

    def index_rows(self, uuid: str):
        n = C.c_int64()
        rc = lib().tfp_group_index_rows(self._h, uuid.encode(), None, None, 0, C.byref(n))
        if rc not in (0, -5):
            self._chk(rc)
        m1 = np.zeros(max(n.value, 1), np.int32)
        m2 = np.zeros(max(n.value, 1), np.int32)
        self._chk(lib().tfp_group_index_rows(self._h, uuid.encode(), m1.ctypes.data, m2.ctypes.data, n.value,
                                             C.byref(n)))
        return m1[:n.value], m2[:n.value]

    def index_stats(self):
        r, c = C.c_int64(), C.c_int32()
        self._chk(lib().tfp_group_index_stats(self._h, C.byref(r), C.byref(c)))
        return r.value, c.value

    def index_commit(self):
        self._chk(lib().tfp_group_index_commit(self._h))

    def search_batch(self, frames: np.ndarray, qoffsets, p: SearchParams):
        frames = np.ascontiguousarray(frames, FRAME_DTYPE)
        qoffsets = np.ascontiguousarray(qoffsets, np.int64)
        nq = len(qoffsets) - 1
        res = (Result * max(1, nq))()
        self._chk(lib().tfp_group_search_batch(self._h, frames.ctypes.data, qoffsets.ctypes.data, nq, C.byref(p), res))
        return Engine._results(res, nq)

    def search_pcm_batch(self, pcm, offsets, p: SearchParams, sample_rate: int = 8000):
        pcm = np.ascontiguousarray(pcm, np.int16)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nq = len(offsets) - 1
        res = (Result * max(1, nq))()
        self._chk(lib().tfp_group_search_pcm_batch(self._h, pcm.ctypes.data, offsets.ctypes.data, nq, sample_rate,
                                                   C.byref(p), res))
        return Engine._results(res, nq)

    def search_f32_batch(self, x, offsets, p: SearchParams, sample_rate: int = 8000):
        x = np.ascontiguousarray(x, np.float32)
        offsets = np.ascontiguousarray(offsets, np.int64)
        nq = len(offsets) - 1
        res = (Result * max(1, nq))()
        self._chk(lib().tfp_group_search_f32_batch(self._h, x.ctypes.data, offsets.ctypes.data, nq, sample_rate,
                                                   C.byref(p), res))
        return Engine._results(res, nq)


class GroupStream:
    """tfp_group_stream: live channels matched against every shard of a Group."""

    def __init__(self, g: Group, nchannels: int, window_samples: int, sample_rate: int = 8000):
        self._g = g
        self._h = C.c_void_p()
        g._chk(lib().tfp_group_stream_create(g.handle, int(nchannels), int(sample_rate), int(window_samples),
                                             C.byref(self._h)))
        self.nchannels = nchannels
        self._res = (Result * nchannels)()
        g._streams.add(self)

    def reset(self, channel: int = -1):
        self._g._chk(lib().tfp_group_stream_reset(self._h, int(channel)))

    def push(self, pcm: np.ndarray, p: SearchParams = None):
        pcm = np.ascontiguousarray(pcm, np.int16)
        assert pcm.shape[0] == self.nchannels
        self._g._chk(lib().tfp_group_stream_push(self._h, pcm.ctypes.data, pcm.shape[1],
                                                 C.byref(p) if p is not None else None,
                                                 self._res if p is not None else None))
        if p is None:
            return None
        return [None if not r.found else {"audio_uuid": r.uuid.decode(), "match_count": r.match_count,
                                          "frame_count": r.frame_count} for r in self._res]

    def close(self):
        if self._h and self._g._h:
            lib().tfp_group_stream_destroy(self._h)
        self._h = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
