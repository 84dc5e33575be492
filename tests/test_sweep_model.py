"""A host model of the coefs=2 sweep's search structures, as tfp_scan.hip builds and reads them:
the window segments' bucket directories filled by the sorted frames' predecessor runs
(wide_bin_sort's dir_runs, with wide_bin_scan's per-segment constants segk), the sweep's bucket
searches (find_ab), and the checkpoint prefix counts (wide_prefix_kernel rows every kPStep frames,
wide_clips' prefix_at). Each is checked against its definition on random segments with crowds of
equal values: the directory entry of bucket b is the first frame whose bucket is >= b, the
searches give the first frame with U2 >= v and the last with L2 <= v, and prefix_at equals the
full in-chunk prefix count. This checks the rules, not the kernels (the -m gpu sweep tests do)."""
import bisect

import numpy as np


def dir_log2(s):
    return 0 if s <= 1 else int(s - 1).bit_length()


def dir_shift(rng, lg):
    bits = int(rng).bit_length() if rng > 0 else 0
    return bits - lg if bits > lg else 0


def segment(rng, n, width):
    """n frames of one window segment sorted by (L2, d): L2 and U2 = L2 + dbase + d both
    non-decreasing (monotone functions of one value, as the frames' max2 bounds are), with crowds."""
    x = np.sort(np.concatenate([rng.integers(-10**6, 10**6, n - n // 3),
                                np.full(n // 3, rng.integers(-10**6, 10**6))]))
    l2 = x // 8
    u2 = (x + 8 * width + 4) // 8
    dbase = width - 3
    d = u2 - l2 - dbase
    assert d.min() >= 0 and d.max() <= 7
    return l2.astype(np.int64), d.astype(np.int64), dbase


def build_dirs(l2, d, sb):
    """wide_bin_scan's constants and dir_runs' writes for the segment's frames at [sb, sb + n)."""
    n = len(l2)
    se = sb + n
    lg = dir_log2(n)
    nbk = 1 << lg
    l2min = int(l2.min())
    shf = dir_shift(int(l2.max()) - l2min + 7, lg)
    tl = np.full(2 * nbk, -1, np.int64)
    for i in range(n):
        bi, bu = (l2[i] - l2min) >> shf, (l2[i] - l2min + d[i]) >> shf
        bp = -1 if i == 0 else (l2[i - 1] - l2min) >> shf
        bq = -1 if i == 0 else (l2[i - 1] - l2min + d[i - 1]) >> shf
        assert bi < nbk and bu < nbk  # (the directory holds every bucket)
        for b in range(bp + 1, bi + 1):
            assert tl[b] == -1
            tl[b] = sb + i
        for b in range(bq + 1, bu + 1):
            assert tl[nbk + b] == -1
            tl[nbk + b] = sb + i
        if i == n - 1:
            for b in range(bi + 1, nbk):
                assert tl[b] == -1
                tl[b] = se
            for b in range(bu + 1, nbk):
                assert tl[nbk + b] == -1
                tl[nbk + b] = se
    assert (tl >= 0).all()  # each bucket written exactly once
    return tl, nbk, shf, l2min


def test_directories_and_searches():
    rng = np.random.default_rng(5)
    for trial in range(300):
        n = int(rng.integers(1, 400))
        width = int(rng.integers(3, 5000))
        l2, d, dbase = segment(rng, n, width)
        u2 = l2 + dbase + d
        sb = int(rng.integers(0, 1000))
        se = sb + n
        tl, nbk, shf, l2min = build_dirs(l2, d, sb)
        u2min = l2min + dbase
        # the definition: entry b = the first frame whose bucket is >= b (se if none)
        bl = (l2 - l2min) >> shf
        bu = (u2 - u2min) >> shf
        for b in range(nbk):
            assert tl[b] == sb + int(np.searchsorted(bl, b, "left"))
            assert tl[nbk + b] == sb + int(np.searchsorted(bu, b, "left"))
        L2s, U2s = list(l2), list(u2)
        pts = np.concatenate([l2, u2, l2 - 1, u2 + 1, rng.integers(l2.min() - 50, u2.max() + 50, 50)])
        for v in pts.tolist():
            # find_ab (tfp_scan.hip wide_clips): B = last L2 <= v, A = first U2 >= v
            dv = v - l2min
            if dv < 0:
                B = sb - 1
            else:
                b = min(dv >> shf, nbk - 1)
                lo, hi = int(tl[b]), int(tl[b + 1]) if b + 1 < nbk else se
                B = lo + bisect.bisect_right(L2s[lo - sb:hi - sb], v) - 1
            du = v - u2min
            if du <= 0:
                A = sb
            else:
                b = min(du >> shf, nbk - 1)
                lo, hi = int(tl[nbk + b]), int(tl[nbk + b + 1]) if b + 1 < nbk else se
                A = lo + bisect.bisect_left(U2s[lo - sb:hi - sb], v)
            assert B == sb + bisect.bisect_right(L2s, v) - 1
            assert A == sb + bisect.bisect_left(U2s, v)


def test_checkpoint_prefix_counts():
    """prefix_at over rows at frames i % 4 == 3 == the full in-chunk prefix, chunks at any
    alignment (QPL = 4: lane l holds queries 4l .. 4l + 3, one byte each)."""
    rng = np.random.default_rng(9)
    step = 4
    for trial in range(40):
        nch = int(rng.integers(1, 6))
        sizes = rng.integers(1, 300, nch)
        cbeg = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int64)
        nf = int(cbeg[-1])
        qis = np.concatenate([rng.integers(0, 256, nf), np.zeros(16, np.int64)])
        full = np.zeros((nf, 256), np.int64)  # in-chunk prefix counts per query
        for ch in range(nch):
            run = np.zeros(256, np.int64)
            for i in range(int(cbeg[ch]), int(cbeg[ch + 1])):
                run[qis[i]] += 1
                full[i] = run
        rows = {i // step: full[i] for i in range(nf) if i % step == step - 1}

        def prefix_at(cb, e):
            g, f0 = e // step, (e // step) * step
            if e == f0 + step - 1:
                return rows[g]
            v = rows[g - 1].copy() if f0 - 1 >= cb else np.zeros(256, np.int64)
            for j in range(step - 1):
                if cb <= f0 + j <= e:
                    v[qis[f0 + j]] += 1
            return v

        for ch in range(nch):
            for e in range(int(cbeg[ch]), int(cbeg[ch + 1])):
                assert (prefix_at(int(cbeg[ch]), e) == full[e]).all()


def seg_max_scan_model(bm, gst):
    """tfp_scan.hip seg_max_scan's DPP steps on 64 lanes: row_shr 1/2/4/8 inside 16-lane rows
    (a lane whose source falls off its row keeps its value), then rows 1 and 3 take lane 15 of the
    row before (row_bcast:15) and rows 2 and 3 lane 31 (row_bcast:31), each step taken only where
    its source lies at or after the lane's group start gst."""
    v = list(bm)
    for n in (1, 2, 4, 8):
        y = [v[l - n] if l % 16 >= n else v[l] for l in range(64)]
        v = [max(v[l], y[l]) if (l % 16 >= n and l - n >= gst[l]) else v[l] for l in range(64)]
    y = [v[(l & ~15) - 1] if (l >> 4) in (1, 3) else v[l] for l in range(64)]
    v = [max(v[l], y[l]) if ((l & 16) and (l & ~15) - 1 >= gst[l]) else v[l] for l in range(64)]
    y = [v[31] if l >= 32 else v[l] for l in range(64)]
    v = [max(v[l], y[l]) if (l >= 32 and 31 >= gst[l]) else v[l] for l in range(64)]
    return v


def test_seg_max_scan_dpp_rule():
    """The run-end scan's DPP form (seg_max_scan) equals its definition, the max of bm over lanes
    [gst, lane] of the lane's group, for random group layouts (wide_clips' batches)."""
    rng = np.random.default_rng(5)
    for _ in range(300):
        cuts = sorted(set([0] + list(rng.integers(1, 64, rng.integers(0, 20)))))
        gst = [max(c for c in cuts if c <= l) for l in range(64)]
        bm = [int(x) for x in rng.integers(-2, 1000, 64)]
        want = [max(bm[gst[l]:l + 1]) for l in range(64)]
        assert seg_max_scan_model(bm, gst) == want


def test_run_queue_ends_equal_serial_closes():
    """wide_clips' run queue (TFP_CLIP_RUNQ): each run's end found lane-parallel (the next start of
    its group, where pe is the running max before it, else its group's last bm) gives the same runs
    [A, end] per group as the serial form that closed the open run at every start and at the group's
    end."""
    rng = np.random.default_rng(9)
    for _ in range(300):
        npts = int(rng.integers(1, 65))
        cuts = sorted(set([0] + list(rng.integers(1, npts, rng.integers(0, 12))) if npts > 1 else [0]))
        ng = len(cuts)
        pj0 = cuts + [npts] * (64 - ng)
        pj1 = cuts[1:] + [npts] + [npts] * (64 - ng)
        gi = [max(j for j in range(ng) if cuts[j] <= l) if l < npts else ng - 1 for l in range(64)]
        gst = [cuts[gi[l]] for l in range(64)]
        A = [int(x) for x in rng.integers(0, 200, 64)]
        B = [a + int(w) - 3 for a, w in zip(A, rng.integers(0, 20, 64))]
        ok = [l < npts and A[l] <= B[l] for l in range(64)]
        bm = [max([B[k] if ok[k] else -2 for k in range(gst[l], l + 1)]) for l in range(64)]
        pe = [-2 if l == gst[l] else bm[l - 1] for l in range(64)]
        starts = [ok[l] and A[l] > pe[l] + 1 for l in range(64)]
        serial = []
        for j in range(ng):
            runs, aopen = [], None
            for l in range(pj0[j], pj1[j]):
                if starts[l]:
                    if aopen is not None:
                        runs.append((aopen, pe[l]))
                    aopen = A[l]
            if aopen is not None:
                runs.append((aopen, bm[pj1[j] - 1]))
            serial.append(runs)
        queued = [[] for _ in range(ng)]
        for l in range(64):
            if not starts[l]:
                continue
            nxt = next((k for k in range(l + 1, 64) if starts[k]), 64)
            gend = pj1[gi[l]]
            end = pe[nxt] if nxt < gend else bm[max(gend - 1, 0)]
            queued[gi[l]].append((A[l], end))
        assert queued == serial


def test_group_mask_equals_binary_lifting():
    """wide_clips' batch groups from the mask of their starts (TFP_CLIP_GROUP_MASK: a lane's group
    = set bits at or below it - 1, its start = the highest such bit, the next group's start = the
    lowest bit above it or the batch's item count) equal the binary lifting over the groups' starts
    pj0 (the last group j < nG with pj0[j] <= lane) for contiguous, non-empty groups."""
    rng = np.random.default_rng(13)
    for _ in range(500):
        npts = int(rng.integers(1, 65))
        cuts = sorted(set([0] + ([int(x) for x in rng.integers(1, npts, rng.integers(0, 20))] if npts > 1 else [])))
        ng = len(cuts)
        pj0 = cuts + [npts] * (64 - ng)
        pj1 = cuts[1:] + [npts] * (65 - ng)
        gm = 0
        for j in range(ng):
            gm |= 1 << pj0[j]
        for lane in range(64):
            gi = 0
            for bit in (32, 16, 8, 4, 2, 1):
                cand = gi + bit
                if cand < ng and pj0[min(cand, 63)] <= lane:
                    gi = cand
            le = (1 << (lane + 1)) - 1
            mgi = bin(gm & le).count("1") - 1
            mgst = (gm & le).bit_length() - 1
            above = gm & ~le & ((1 << 64) - 1)
            mgend = (above & -above).bit_length() - 1 if above else npts
            assert (mgi, mgst, mgend) == (gi, pj0[gi], pj1[gi]), (lane, cuts)
