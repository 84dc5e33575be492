"""The fp_handler mirror on the GPU: the batched directory enrolment (app_tiresias.c:365-424)
enrols exactly what per-file fp_craete_audio_list_info calls enrol, and search finds it."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _write_dir(tfp_lib, d):
    from tiresias_amd.fp_handler import write_wav_mono16
    os.makedirs(d, exist_ok=True)
    pcm = tfp_lib.synth_pcm(0x7153A1, range(5), 40000)
    for i in range(5):
        write_wav_mono16(os.path.join(d, "clip%02d.wav" % i), pcm[i])
    write_wav_mono16(os.path.join(d, "dup_of_clip01.wav"), pcm[1])            # same MD5: enrolled once
    write_wav_mono16(os.path.join(d, "short.wav"), pcm[2][:300])              # 2 frames
    write_wav_mono16(os.path.join(d, "clip16k.wav"), pcm[3][:32000], 16000)   # another rate
    with open(os.path.join(d, "notes.txt"), "w") as f:                          # not a WAV: skipped
        f.write("not audio")
    return pcm


def test_directory_enrolment_equals_per_file(tfp_lib, tmp_path):
    from tiresias_amd import FpHandler
    d = str(tmp_path / "lib")
    pcm = _write_dir(tfp_lib, d)
    a = FpHandler(0)
    b = FpHandler(0)
    assert a.fp_init() and b.fp_init()
    try:
        for h in (a, b):
            assert h.fp_create_context_list_info("ctx", d, False)
        assert a.create_new_audio_info("ctx")
        for name in sorted(os.listdir(d)):
            b.fp_craete_audio_list_info("ctx", os.path.join(d, name))
        ra = sorted((r["name"], r["hash"]) for r in a.fp_get_audio_lists_all())
        rb = sorted((r["name"], r["hash"]) for r in b.fp_get_audio_lists_all())
        assert ra == rb and len(ra) == 7  # 5 clips + short + 16 kHz; the duplicate and the .txt skipped
        ua = {r["name"]: r["uuid"] for r in a.fp_get_audio_lists_all()}
        ub = {r["name"]: r["uuid"] for r in b.fp_get_audio_lists_all()}
        for name in ua:
            m1a, m2a = a.engine.index_rows(ua[name])
            m1b, m2b = b.engine.index_rows(ub[name])
            assert np.array_equal(m1a, m1b) and np.array_equal(m2a, m2b), name
        # a second scan enrols nothing new
        assert a.create_new_audio_info("ctx")
        assert len(a.fp_get_audio_lists_all()) == 7
        # search an excerpt of clip03 through the mirror
        q = str(tmp_path / "q.wav")
        from tiresias_amd.fp_handler import write_wav_mono16
        write_wav_mono16(q, pcm[3][256 * 10: 256 * 10 + 24000])
        for tol in (0.45, 0.001):
            res_a = a.fp_search_fingerprint_info("ctx", q, 1, tol, -1, -1)
            res_b = b.fp_search_fingerprint_info("ctx", q, 1, tol, -1, -1)
            # uuids are random per handler and ties go to the greatest uuid: compare the counts
            key = lambda r: None if r is None else (r["match_count"], r["frame_count"])  # noqa: E731
            assert key(res_a) == key(res_b)
        assert res_a is None or res_a["frame_count"] == 94
    finally:
        a.fp_term()
        b.fp_term()


def test_directory_enrolment_bad_context(tfp_lib, tmp_path):
    from tiresias_amd import FpHandler
    h = FpHandler(0)
    assert h.fp_init()
    try:
        assert not h.create_new_audio_info("nope")
        assert h.fp_create_context_list_info("c2", str(tmp_path / "missing"), False)
        assert not h.create_new_audio_info("c2")
    finally:
        h.fp_term()


def test_stereo_and_24bit_enrolment_through_fp32_path(tfp_lib, oracle, tmp_path):
    """Files the int16 ingest refuses (stereo 16-bit, 24-bit) are enrolled through
    tfp_wav_read_f32 + tfp_fingerprint_f32_batch; stored rows equal the oracle's fingerprints of
    aubio's fp32 source values; the mirror's search reads them the same way."""
    import struct
    from tiresias_amd import FpHandler
    pcm = tfp_lib.synth_pcm(0x7153A1, [1, 2], 40000)

    def riff(ch, bits, data):
        align = ch * bits // 8
        fmt = struct.pack("<HHIIHH", 1, ch, 8000, 8000 * align, align, bits)
        body = b"WAVE" + b"fmt " + struct.pack("<I", 16) + fmt + b"data" + struct.pack("<I", len(data)) + data
        return b"RIFF" + struct.pack("<I", len(body)) + body

    d = tmp_path / "st"
    d.mkdir()
    st = np.stack([pcm[0], pcm[1]], 1)
    (d / "a_stereo.wav").write_bytes(riff(2, 16, st.astype("<i2").tobytes()))
    x24 = (pcm[0].astype(np.int64) << 8) + np.arange(40000) % 256
    u = x24 & 0xFFFFFF
    (d / "b_24bit.wav").write_bytes(riff(1, 24, np.stack([u & 255, (u >> 8) & 255, u >> 16], 1).astype(np.uint8).tobytes()))
    want = {"a_stereo.wav": oracle.wav_mono_f32(st, 16), "b_24bit.wav": oracle.wav_mono_f32(x24[:, None], 24)}
    h = FpHandler(0)
    assert h.fp_init()
    try:
        assert h.fp_create_context_list_info("ctx", str(d), False)
        assert h.create_new_audio_info("ctx")
        rows = {r["name"]: r["uuid"] for r in h.fp_get_audio_lists_all()}
        assert sorted(rows) == sorted(want)
        for name, x in want.items():
            m1, m2 = h.engine.index_rows(rows[name])
            _, _, micro = oracle.fingerprint_f32(x)
            assert np.array_equal(m1, micro[:, 0]) and np.array_equal(m2, micro[:, 1]), name
        # the mirror's search of the stereo file = the oracle's fp_search_fingerprint_info over the
        # enrolled rows, with the query's fp32 fingerprints
        names = sorted(want)
        uuids = [rows[n] for n in names]
        mic = [oracle.fingerprint_f32(want[n])[2] for n in names]
        m1 = np.concatenate([m[:, 0] for m in mic])
        m2 = np.concatenate([m[:, 1] for m in mic])
        clip = np.concatenate([np.full(len(m), i, np.int32) for i, m in enumerate(mic)])
        _, qdb, _ = oracle.fingerprint_f32(want["a_stereo.wav"])
        for tol in (0.45, 0.001):
            res = h.fp_search_fingerprint_info("ctx", str(d / "a_stereo.wav"), 1, tol, -1, -1)
            found, w, mc, fc = oracle.search(m1, m2, clip, uuids, qdb[:, 0], qdb[:, 1], 1, tol)
            assert (res is not None) == found
            if found:
                assert (res["uuid"], res["match_count"], res["frame_count"]) == (uuids[w], mc, fc) == (uuids[w], mc, 157)
    finally:
        h.fp_term()
