#!/usr/bin/env python3
"""Debug helper (test infrastructure): prints the reference's and the restatement's PUSCH channel estimates side by
side for one random case. Usage: python tools/debug/chest_compare.py [seed] [nof_rb]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402

import pusch_chest_oracle as C  # noqa: E402
from ofdm_oracle import bf16_to_complex  # noqa: E402
from oracle_lib import Reference  # noqa: E402
from pusch_chest_cases import random_case  # noqa: E402

seed = int(sys.argv[1]) if len(sys.argv) > 1 else 401
nrb = int(sys.argv[2]) if len(sys.argv) > 2 else 2
ref = Reference()
rng = np.random.default_rng(seed)
cfg, grid, H = random_case(rng, 24, nof_rb=nrb, dmrs_type2=0)
ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid, 24)
ch, nvo, rsrpo, epreo, _ = C.estimate(cfg, bf16_to_complex(grid), "filter")
got = bf16_to_complex(ce)
np.set_printoptions(precision=3, linewidth=220)
r0 = cfg["rb_start"] * 12
print(cfg)
l = cfg["start_symbol"]
print("ref ", got[0, l, r0:r0 + 24])
print("orc ", ch[0, l, r0:r0 + 24])
print("true", H[0, r0:r0 + 24])
print("ref nonzero symbols", np.nonzero(np.abs(got[0]).sum(1))[0])
print("ref nonzero sc", np.nonzero(np.abs(got[0]).sum(0))[0][[0, -1]])
