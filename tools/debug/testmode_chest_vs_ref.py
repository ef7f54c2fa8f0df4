#!/usr/bin/env python3
"""Diagnostic (GPU box): the test-mode UL slot (one 273-PRB UE, DM-RS 2 + 11) synthesized exactly as the bench does,
OFDM-demodulated by the GPU; then the GPU estimator's noise variance / SNR / TA / CFO next to the reference estimator's
(oracle/_ref/libsrsref.so, test infrastructure) on the very same received grid, per rx port. Also the post-equalisation
SINR of the GPU demodulator. A checker, not part of the product path."""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import srsgpu  # noqa: E402
from srsgpu import slot as slotlib  # noqa: E402
from oracle_lib import Reference  # noqa: E402
import pusch_chest_oracle as C  # noqa: E402
from ofdm_oracle import bf16_to_complex  # noqa: E402

ref = Reference()
ctx = srsgpu.Context(0)
gen = torch.Generator(device="cuda")
gen.manual_seed(3)
_, _, ul_cell = slotlib.tdd_testmode_cells(1)
ul = slotlib.UplinkPipeline(ctx, ul_cell, equalizer=srsgpu.EQ_ZF, estimate_layout=srsgpu.CE_PER_SYMBOL)
sent = torch.randint(0, 256, (sum(ul.tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
for snr in (26.0, 30.0):
    x = slotlib.synthesize_uplink(ctx, ul_cell, sent, snr_db=snr, seed=99, cfo_hz_max=300.0)
    ul.execute(x, torch.cuda.current_stream())
    torch.cuda.synchronize()
    nsc = ul_cell.nsc
    grid = ul.d_grid.cpu().numpy().view(np.uint16).reshape(ul_cell.nof_slots, 4, 14, nsc, 2)
    m = ul.d_metrics.cpu().numpy().reshape(-1, 4, srsgpu.CHEST_METRICS)
    ce_gpu = ul.d_ce.cpu().numpy().view(np.uint16).reshape(ul_cell.nof_slots, 4, 4, 14, nsc, 2)
    for s in range(ul_cell.nof_slots):
        cfg = dict(slot=ul_cell.slot_index(s), scrambling_id=500, n_scid=0, dmrs_type2=0, scaling=slotlib.DMRS_BETA,
                   dmrs_symbol_mask=ul_cell.dmrs_mask, start_symbol=0, nof_symbols=14, rb_start=0, nof_rb=273,
                   nof_rx_ports=4)
        ce, nv, rsrp, epre, ta, cfo = ref.pusch_chest(cfg, grid[s], 273, fd=2, td=0, compensate_cfo=True)
        ch_o, nv_o, rsrp_o, _, ex = C.estimate(cfg, bf16_to_complex(grid[s]), "filter", "average", True)
        g_ce = bf16_to_complex(ce_gpu[s, 0])[:, 0]
        r_ce = bf16_to_complex(ce)[:, 0]
        err = np.abs(g_ce - r_ce).max() / np.sqrt(np.mean(np.abs(r_ce) ** 2))
        print(f"snr {snr} slot {s}: ref nv {nv} snr_dB {10 * np.log10(rsrp / cfg['scaling'] ** 2 / nv).round(2)}"
              f" ta {ta} cfo {cfo}", flush=True)
        print(f"   oracle nv {nv_o} ta {ex['ta_s']} cfo {ex['cfo_hz']}")
        print(f"   gpu    nv {m[s, :, 2]} snr_dB {(10 * np.log10(m[s, :, 3])).round(2)} ta {m[s, :, 4]} "
              f"cfo {m[s, :, 5]} rsrp {m[s, :, 0]} (ref {rsrp}); estimate row-0 max err / rms {err:.3e}", flush=True)
    print(f"   tb_ok {ul.d_tb_ok.cpu().numpy().tolist()} cb_ok {ul.d_crc.cpu().numpy().mean():.3f}", flush=True)
