"""Live channels (configs[4] semantics): after every tick, each channel's result equals the
reference search on a recording of that channel's most recent window (the WAV the dialplan
app records, application_handler.c:248-312)."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SEED_DB = 0x7153A1


def test_stream_equals_oracle_on_last_window(engine, oracle, tfp_lib):
    from tiresias_amd import Stream
    nclips, n = 40, 8000 * 8
    pcm = tfp_lib.synth_pcm(SEED_DB, range(nclips), n)
    micro, _ = oracle.fingerprint_batch(pcm.reshape(-1), np.arange(nclips + 1) * n, nthreads=8, want_db=False)
    nf = (n + 255) // 256
    uuids = ["%08x-1111-4000-8000-%012x" % (c * 2654435761 % 2**32, c) for c in range(nclips)]
    engine.index_clear()
    for c in range(nclips):
        engine.index_add(uuids[c], micro[c * nf:(c + 1) * nf, 0], micro[c * nf:(c + 1) * nf, 1])
    clip = np.repeat(np.arange(nclips), nf)

    nch, W, T = 6, 8000 * 2, 160  # 2 s windows, 20 ms SLIN ticks
    st = Stream(engine, nch, W)
    p = tfp_lib.params(1, 0.45)
    # channels play excerpts of enrolled clips (ch 5: unrelated audio); ch 2 starts a new call midway
    src = [tfp_lib.synth_pcm(SEED_DB, [3 * c + 1], 8000 * 6, offsets=[1000 * c])[0] for c in range(5)]
    src.append(tfp_lib.synth_pcm(0xBEEF, [0], 8000 * 6)[0])
    hist = [[] for _ in range(nch)]
    checked = 0
    for tick in range(250):
        blk = np.stack([s[tick * T:(tick + 1) * T] for s in src])
        if tick == 150:
            st.reset(2)
            hist[2] = []
        for c in range(nch):
            hist[c].append(blk[c])
        res = st.push(blk, p if tick % 7 == 0 or tick == 249 else None)
        if res is None:
            continue
        for c in range(nch):
            h = np.concatenate(hist[c]) if hist[c] else np.zeros(0, np.int16)
            if len(h) < W:
                assert res[c] is None
                continue
            win = h[-W:]
            _, qdb, _ = oracle.fingerprint(win)
            found, w, mc, fc = oracle.search(micro[:, 0], micro[:, 1], clip, uuids, qdb[:, 0], qdb[:, 1], 1, 0.45, -1, -1)
            exp = (uuids[w], mc, fc) if found else None
            got = None if res[c] is None else (res[c]["audio_uuid"], res[c]["match_count"], res[c]["frame_count"])
            assert got == exp, (tick, c)
            checked += 1
    assert checked > 60
    engine.index_clear()
