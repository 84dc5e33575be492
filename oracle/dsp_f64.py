"""Float64 numpy restatement of the per-hop DSP (test infrastructure only).

Independent cross-check of the C oracle's arithmetic structure: the same aubio tables
(window, Slaney filterbank, DCT rows; built by the oracle from the aubio 0.4.5 expressions)
applied with numpy's float64 real FFT. Agreement is within float32 rounding, which proves
the oracle's canonical 16x16 FFT is a correct 512-point DFT and that framing / fftshift /
filterbank / log / DCT are wired as /root/reference/src/fp_handler.c:632-652 + libaubio do.
"""
from __future__ import annotations

import numpy as np


def fingerprint_f64(pcm: np.ndarray, tabs: dict) -> np.ndarray:
    """-> coef float64[F, 2] (MFCC c0, c1) for one clip."""
    x = pcm.astype(np.float64) / 32768.0
    nf = (len(x) + 255) // 256
    padded = np.zeros((nf + 1) * 256, np.float64)
    padded[256:256 + len(x)] = x            # one zero hop of history before frame 0
    w = tabs["window"].astype(np.float64)
    mel = tabs["mel"].astype(np.float64)
    dct = tabs["dct"].astype(np.float64)
    out = np.zeros((nf, 2), np.float64)
    for f in range(nf):
        data = padded[f * 256:f * 256 + 512] * w
        data = np.concatenate([data[256:], data[:256]])  # fvec_shift
        norm = np.abs(np.fft.rfft(data))
        band = mel @ norm
        logb = np.log10(np.maximum(2e-42, band))
        out[f] = dct @ logb
    return out
