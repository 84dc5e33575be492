"""LDS bank-conflict model of the fingerprint kernel's per-pass accesses (one wave, 64 lanes =
4 frames x 16 lanes), following MI355X_MICROARCH.md §LDS: per instruction the lane groups and
the bank function; identical addresses broadcast; N distinct addresses on a bank in a group
cost N cycles. Prints extra (conflict) cycles per pass and per access kind.
Usage: python scripts/tools/lds_banks.py [frame_stride_float2] [hop_stride_samples]"""
import sys

sys.path.insert(0, ".")
FS = int(sys.argv[1]) if len(sys.argv) > 1 else 258
HS = int(sys.argv[2]) if len(sys.argv) > 2 else 288
PAD = len(sys.argv) > 3 and sys.argv[3] == "pad17"  # padded square W[L*17 + k] instead of XOR swizzle
NOFF = 16 if PAD else 0                                 # |X| row of odd frames shifted by 16 floats

G_B32 = [list(range(0, 32)), list(range(32, 64))]
G_B128 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)],
          [*range(32, 36), *range(44, 48), *range(52, 60)], [*range(36, 44), *range(48, 52), *range(60, 64)]]
G_W64 = [list(range(16 * i, 16 * i + 16)) for i in range(4)]
G_W128 = [list(range(8 * i, 8 * i + 8)) for i in range(8)]
KIND = {  # instruction -> (groups, dwords per lane, bank modulus, ideal cycles)
    "ds_read_b32": (G_B32, 1, 32), "ds_read_b64": (G_B32, 2, 64), "ds_read_b128": (G_B128, 4, 64),
    "ds_write_b32": (G_B32, 1, 32), "ds_write_b64": (G_W64, 2, 32), "ds_write_b128": (G_W128, 4, 32)}


def extra(ins, addr):
    """addr[lane] = byte address or None (inactive). Returns extra cycles beyond one per group."""
    groups, dw, mod = KIND[ins]
    ex = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addr[l]
            if a is None:
                continue
            for d in range(dw):
                b = (a // 4 + d) % mod
                banks.setdefault(b, set()).add(a // 4 + d)
        if banks:
            ex += max(len(v) for v in banks.values()) - 1
    return ex


def lanes():
    return [(l >> 4, l & 15) for l in range(64)]


def main():
    import ctypes  # noqa: F401
    tot = {}
    # PCM staging (ds_write_b128), 3 rounds of 64 chunks
    for r in range(3):
        ad = []
        for l in range(64):
            ch = l + 64 * r
            ad.append(((ch >> 5) * HS + (ch & 31) * 8) * 2 if ch < 160 else None)
        tot["pcm stage w128"] = tot.get("pcm stage w128", 0) + extra("ds_write_b128", ad)
    # PCM reads (ds_read_b32) z[n1]
    for n1 in range(16):
        hsel = 1 if n1 < 8 else 0
        ad = [((g * HS + hsel * HS + (((32 * n1 + 2 * L + 256) & 511) & 255)) * 2) for g, L in lanes()]
        tot["pcm read b32"] = tot.get("pcm read b32", 0) + extra("ds_read_b32", ad)
    pcm_base = 0
    # transpose write b64 / read b64
    for k1 in range(16):
        ad = [(g * FS + (L * 17 + k1 if PAD else L * 16 + (k1 ^ L))) * 8 for g, L in lanes()]
        tot["transpose w64"] = tot.get("transpose w64", 0) + extra("ds_write_b64", ad)
    for n2 in range(16):
        ad = [(g * FS + (n2 * 17 + L if PAD else n2 * 16 + (L ^ n2))) * 8 for g, L in lanes()]
        tot["transpose r64"] = tot.get("transpose r64", 0) + extra("ds_read_b64", ad)
    # |X| writes b32
    for k2 in range(16):
        ad = [(g * FS * 2 + NOFF * (g & 1) + L + 16 * k2) * 4 for g, L in lanes()]
        tot["N write b32"] = tot.get("N write b32", 0) + extra("ds_write_b32", ad)
    # filterbank: |X| b128 reads + weight b128 reads (8 kHz slot schedule from the host tables)
    try:
        import numpy as np  # noqa: F401
        sched = slot_schedule()
    except Exception as e:  # pragma: no cover
        print("no schedule:", e)
        sched = None
    if sched:
        lens, starts = sched
        for sl in range(3):
            for q in range(0, lens[sl], 4):
                ad = [(g * FS * 2 + NOFF * (g & 1) + starts[sl][L] + q) * 4 for g, L in lanes()]
                tot["mel N r128"] = tot.get("mel N r128", 0) + extra("ds_read_b128", ad)
                ad = [(16 * q + 4 * L) * 4 for g, L in lanes()]
                tot["mel w r128 (interleaved)"] = tot.get("mel w r128 (interleaved)", 0) + extra("ds_read_b128", ad)
                ad = [(L * lens[sl] + q) * 4 for g, L in lanes()]
                tot["mel w r128 (per-lane rows)"] = tot.get("mel w r128 (per-lane rows)", 0) + extra("ds_read_b128", ad)
    print(f"frame stride {FS} float2, hop stride {HS} samples, {'padded' if PAD else 'xor'} square:"
          " extra LDS cycles per pass")
    for k, v in tot.items():
        print(f"  {k:28s} {v}")


def slot_schedule():
    """8 kHz slot lengths/starts via the engine's table dump helper (tests/native/dump_tables)."""
    import subprocess
    import os
    exe = "/tmp/tfp_slots"
    src = "/tmp/tfp_slots.cpp"
    open(src, "w").write('#include "tfp_tables.hpp"\n#include <cstdio>\nusing namespace tfp;\nint main(){static DspTables t;'
                         'build_tables(8000,&t);for(int s=0;s<3;s++){printf("%d",t.ms_len[s]);for(int L=0;L<16;L++)'
                         'printf(" %d",t.ms_start[s][L]);printf("\\n");}}\n')
    root = os.path.abspath(".")
    subprocess.check_call(["g++", "-O1", "-std=c++17", "-fno-builtin", "-ffp-contract=off",
                           f"-I{root}/asterisk-tiresias_amd/csrc", f"-I{root}/include", src,
                           f"{root}/asterisk-tiresias_amd/csrc/tfp_tables.cpp", "-o", exe])
    rows = [list(map(int, l.split())) for l in subprocess.check_output([exe]).decode().split("\n") if l.strip()]
    return [r[0] for r in rows], [r[1:] for r in rows]


if __name__ == "__main__":
    main()
