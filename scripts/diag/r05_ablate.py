"""Diagnostic (not product code): build ablated copies of the library for a phase-cost study of
fingerprint8k_kernel<4>. Each variant removes one piece of a pass (its results are WRONG on
purpose) so that the C2 launch time with and without it bounds what that piece costs.

usage: python scripts/diag/r05_ablate.py NAME [NAME ...]   (or "all")
Writes asterisk-tiresias_amd/abv/<NAME>/libtiresias_fp.so; time them with scripts/diag/fp_c2.py
(TFP_LIB_PATH=...). The patched sources live only in a temporary copy of the committed tree (git HEAD).
"""
import os
import shutil
import subprocess
import sys
import tempfile

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
PKG = os.path.join(REPO, "asterisk-tiresias_amd")

K = "csrc/tfp_kernels.hip"
SP = "csrc/tfp_split.hpp"
SC = "csrc/tfp_scan.hip"
ABL = {
    "base": [],
    # raw v_sqrt_f32, no Tuckerman correction
    "nosqrtfix": [(SP, "  step_tuckerman(m0, m1, rp, rm, n0, n1);",
                   "  (void)rp; (void)rm; (void)m0; (void)m1; n0 = __builtin_bit_cast(float, b0); n1 = __builtin_bit_cast(float, b1);")],
    # window and split twiddles from registers-free constants (no 16 b128 LDS reads per pass)
    "noconst": [(K, "const float4 w4 = *reinterpret_cast<const float4*>(winr + (i * 16 + L) * 2 + oz);",
                 "const float4 w4 = make_float4(1.f + i, 0.5f, 0.25f * L, 3.f);"),
                (K, "const float4 t4 = tw4[16 * k2];",
                 "const float4 t4 = make_float4(0.1f * k2, 0.2f, 0.3f * L, 0.7f); (void)tw4;")],
    # no band logs in the tile tail
    "nologs": [(K, "const float l = log_finish(g[r], en[r]);", "const float l = g[r].m + (float)(en[r].invc > 0);")],
    # no frame-pair filterbank
    "nofb": [(K, "if (sub == 1) pair_fb(std::integral_constant<int, 0>{});\n        else pair_fb(std::integral_constant<int, 1>{});",
              "(void)pair_fb;")],
    # no rare-bin test
    "norare": [(K, "umin = min(umin, rare_key_pair(sq));", "(void)umin;")],
    # transposes without LDS (each lane keeps its own values)
    "notrans": [(K, """#pragma unroll
        for (int k1 = 0; k1 < 16; k1++) W[k1 * kSq8 + L] = Y[k1];
        wave_sync();
#pragma unroll
        for (int n2 = 0; n2 < 16; n2 += 2) {
          const float4 v = *reinterpret_cast<const float4*>(W + L * kSq8 + n2);
          z[n2] = cf{v.x, v.y};
          z[n2 + 1] = cf{v.z, v.w};
        }""", """#pragma unroll
        for (int n2 = 0; n2 < 16; n2++) z[n2] = Y[n2];""")],
    # partner exchange without ds_bpermute
    "nobperm": [(K, "Pq[k2] = cf{partner16(Y[15 - k2].x), partner16(Y[15 - k2].y)};", "Pq[k2] = Y[15 - k2];")],
    # coefs=2 bin sort (tfp_scan.hip wide_bin_sort) without its sorts: the groups written unsorted,
    # and info[2] set so the directory fill and the sweep skip the batch (it is redone with the
    # library sort): only the kernel's own duration in a trace means anything
    "binsort_nosort": [(SC, "    bitonic_regs<R>(v, lane);\n", "\n"),
                       (SC, "    bitonic_lds(S, N, lane);\n", "\n"),
                       (SC, "  const int32_t* bs = bstart + (int64_t)ch * (kNFine + 1);\n  if (g + 1 >= gcap) return;",
                        "  const int32_t* bs = bstart + (int64_t)ch * (kNFine + 1);\n"
                        "  if (blockIdx.x == 0 && blockIdx.y == 0 && threadIdx.x == 0) atomicAdd(&info[2], 1);\n"
                        "  if (g + 1 >= gcap) return;")],
}


def build(name):
    edits = ABL[name]
    tmp = tempfile.mkdtemp(prefix=f"abl_{name}_")
    try:
        # the committed tree (HEAD), not the working copy
        subprocess.run(f"git -C {REPO} archive HEAD asterisk-tiresias_amd include | tar -x -C {tmp}", shell=True, check=True)
        dst = os.path.join(tmp, "asterisk-tiresias_amd")
        for f, a, b in edits:
            p = os.path.join(dst, f)
            s = open(p).read()
            if s.count(a) != 1:
                sys.exit(f"{name}: pattern not found once in {f}: {a[:60]!r}")
            open(p, "w").write(s.replace(a, b))
        subprocess.run(["make", "-s", "-j8", "lib/libtiresias_fp.so"], cwd=dst, check=True)
        out = os.path.join(PKG, "abv", name)
        os.makedirs(out, exist_ok=True)
        shutil.copy(os.path.join(dst, "lib", "libtiresias_fp.so"), out)
        print("built", out)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    names = list(ABL) if sys.argv[1:] == ["all"] else sys.argv[1:]
    for n in names:
        build(n)
