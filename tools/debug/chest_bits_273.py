#!/usr/bin/env python3
"""Diagnostic (GPU box, test infrastructure): where do the GPU's 273-PRB channel estimates and the reference's differ
by a bf16 ulp? On the GPU's own OFDM-demodulated grid (so only the estimator differs), with and without CFO
compensation, classify the differing estimate words: a whole row (every symbol of a (port, subcarrier) differs: the
smoothed estimate itself) or single symbols (the per-symbol CFO rotation), and print the CFO bits of both.
Usage: python tools/debug/chest_bits_273.py"""
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


def main():
    ref = Reference()
    ctx = srsgpu.Context(0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234)
    _, _, cell = slotlib.tdd_testmode_cells(1)
    nsc, S = cell.nsc, cell.nof_slots
    pipes = {cfo: slotlib.UplinkPipeline(ctx, cell, equalizer=srsgpu.EQ_ZF, estimate_layout=srsgpu.CE_PER_SYMBOL,
                                         compensate_cfo=cfo) for cfo in (True, False)}
    sent = torch.randint(0, 256, (sum(pipes[True].tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
    for snr in (30.0, 26.0):
        for seed in (99, 1099):
            x = slotlib.synthesize_uplink(ctx, cell, sent, snr_db=snr, seed=seed, cfo_hz_max=300.0)
            for cfo, ul in pipes.items():
                ul.execute(x, torch.cuda.current_stream())
                torch.cuda.synchronize()
                grid_all = ul.d_grid.cpu().numpy().view(np.uint16).reshape(S, 4, 14, nsc, 2)
                ce_all = ul.d_ce.cpu().numpy().view(np.uint32).reshape(S, 4, 4, 14, nsc)
                m = ul.d_metrics.cpu().numpy().reshape(-1, 4, srsgpu.CHEST_METRICS)
                for s in range(S):
                    ccfg = dict(slot=cell.slot_index(s), scrambling_id=500, n_scid=0, dmrs_type2=0,
                                scaling=slotlib.DMRS_BETA, dmrs_symbol_mask=cell.dmrs_mask, start_symbol=0,
                                nof_symbols=14, rb_start=0, nof_rb=273, nof_rx_ports=4)
                    rce, rnv, rrsrp, _, _, rcfo = ref.pusch_chest(ccfg, grid_all[s], 273, fd=2, td=0,
                                                                  compensate_cfo=cfo)
                    rw = rce.view(np.uint32)[..., 0]      # (P, 14, nsc)
                    gw = ce_all[s, 0]                     # layer 0: (P, 14, nsc)
                    diff = gw != rw
                    per_sc = diff.sum(axis=1)             # (P, nsc): symbols differing per (port, sc)
                    rows = int(np.sum(per_sc == 14))
                    partial = int(np.sum((per_sc > 0) & (per_sc < 14)))
                    print(f"snr {snr} seed {seed} cfo_comp {cfo} slot {s}: words differing {int(diff.sum())}; "
                          f"(port, sc) rows all-14 {rows}, partial {partial}; "
                          f"cfo gpu {m[s, :, 5].view(np.uint32)} ({m[s, :, 5]}) ref {rcfo.view(np.uint32)} ({rcfo}); "
                          f"nv bits equal {np.array_equal(m[s, :, 2].view(np.uint32), rnv.view(np.uint32))}",
                          flush=True)
                    if cfo:
                        for p, k in list(zip(*np.nonzero((per_sc > 0) & (per_sc < 14))))[:3]:
                            syms = np.nonzero(diff[p, :, k])[0]
                            print(f"    partial p{p} sc{k}: symbols {syms.tolist()} gpu "
                                  f"{[hex(v) for v in gw[p, syms, k]]} ref {[hex(v) for v in rw[p, syms, k]]}",
                                  flush=True)
                        for p, k in list(zip(*np.nonzero(per_sc == 14)))[:3]:
                            print(f"    row p{p} sc{k} (rb {k // 12} re {k % 12}): gpu {hex(gw[p, 0, k])} ref "
                                  f"{hex(rw[p, 0, k])}", flush=True)


if __name__ == "__main__":
    main()
