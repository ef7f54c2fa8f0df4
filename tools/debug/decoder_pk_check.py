"""Debug helper: per-(BG, Z) parity of the GPU decoder against the oracle, printing every mismatch (no early exit)."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))
import torch  # noqa: E402,F401
import srsgpu  # noqa: E402
from oracle_lib import BG_K, BG_N_SHORT, CRC24B, LIFTING_SIZES, Oracle, encode_with_llrs  # noqa: E402


def main():
    orc = Oracle()
    ctx = srsgpu.Context(0)
    rng = np.random.default_rng(7)
    for mode, name in ((1, "avx2"), (0, "generic")):
        dec = srsgpu.LdpcDecoder(ctx, name)
        for bg in (1, 2):
            bad = []
            for Z in [z for z in LIFTING_SIZES if BG_K[bg] * z >= 48]:
                for max_iter, use_crc in ((1, False), (3, False), (8, True)):
                    K, N = BG_K[bg], BG_N_SHORT[bg]
                    _, _, llr = encode_with_llrs(orc, rng, bg, Z, crc_poly=CRC24B, nof_filler=0, amp=12, noise=8.0,
                                                 n_llr=N * Z)
                    cfg = srsgpu.CodeblockDecodeConfig(bg, Z, nof_crc_bits=24, nof_filler_bits=0,
                                                       max_iterations=max_iter)
                    r, bits = orc.ldpc_decode(mode, bg, Z, llr, nof_crc_bits=24, nof_filler=0,
                                              crc_poly=CRC24B if use_crc else -1, max_iter=max_iter, scaling=0.8)
                    (rg, bg_bits), = dec.decode_batch([llr], [cfg], [CRC24B if use_crc else None])
                    ok = (rg == (None if r < 0 else r)) and np.array_equal(bg_bits, bits)
                    if not ok:
                        nd = int(np.count_nonzero(bg_bits != bits))
                        bad.append((Z, max_iter, use_crc, rg, r, nd))
            print(name, "BG", bg, "mismatches:", len(bad), bad[:12], flush=True)


if __name__ == "__main__":
    main()
