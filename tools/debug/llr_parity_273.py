#!/usr/bin/env python3
"""Diagnostic (GPU box, test infrastructure): where do the GPU's UL LLRs and the reference's differ on 273-PRB slots?

For the test-mode UL slots (one 273-PRB UE, DM-RS 2 + 11, ZF 1x4, CFO compensation), synthesised like the bench, the
chain is split at every stage boundary and the reference (oracle/_ref/libsrsref.so) is run on the GPU's intermediate
results, so each stage's contribution to an LLR difference is isolated:

  A  GPU chain (OFDM demod -> estimator -> demodulator)               vs  B  reference chain on the same samples
  C  GPU grid vs reference grid (OFDM demodulator only)
  D  reference estimator + demodulator on the GPU's grid              vs  A   (estimator + demodulator)
  E  reference demodulator on the GPU's grid, estimates and nv        vs  A   (demodulator only)
  F  reference demodulator on the GPU's grid + reference estimates    vs  D   (estimates only)

For every LLR that differs by more than one step, the RE (symbol, subcarrier), both estimates, both grids and the
equalised symbol are printed. Usage: python tools/debug/llr_parity_273.py [snr_db ...]"""
import ctypes
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
from ofdm_oracle import bf16_to_complex  # noqa: E402

P_ = ctypes.c_void_p


def stats(a, b):
    d = np.abs(a.astype(np.int16) - b.astype(np.int16))
    return dict(n=int(d.size), equal=float(np.mean(d == 0)), within1=float(np.mean(d <= 1)), max=int(d.max()),
                over1=int(np.sum(d > 1)))


def main():
    snrs = [float(x) for x in sys.argv[1:]] or [30.0, 26.0, 35.0]
    ref = Reference()
    lib = ref.lib
    lib.ref_ul_slot_timed_at.restype = ctypes.c_longlong
    ctx = srsgpu.Context(0)
    gen = torch.Generator(device="cuda")
    gen.manual_seed(1234)
    _, _, cell = slotlib.tdd_testmode_cells(1)
    nsc, S = cell.nsc, cell.nof_slots
    data_syms = [l for l in range(14) if not (cell.dmrs_mask >> l) & 1]
    out = {"compact": {}, "per_symbol": {}}
    pipes = {name: slotlib.UplinkPipeline(ctx, cell, equalizer=srsgpu.EQ_ZF, estimate_layout=lay, compensate_cfo=True)
             for name, lay in (("compact", srsgpu.CE_COMPACT), ("per_symbol", srsgpu.CE_PER_SYMBOL))}
    sent = torch.randint(0, 256, (sum(pipes["compact"].tb_bytes),), generator=gen, device="cuda", dtype=torch.uint8)
    qm = cell.ues[0].qm
    for snr in snrs:
        for seed in (99, 1099, 2099):
            x = slotlib.synthesize_uplink(ctx, cell, sent, snr_db=snr, seed=seed, cfo_hz_max=300.0)
            res = {}
            for name, ul in pipes.items():
                ul.execute(x, torch.cuda.current_stream())
                torch.cuda.synchronize()
                res[name] = ul.d_llrs.cpu().numpy().copy()
            ul = pipes["per_symbol"]
            grid_all = ul.d_grid.cpu().numpy().view(np.uint16).reshape(S, 4, 14, nsc, 2)
            ce_all = ul.d_ce.cpu().numpy().view(np.uint16).reshape(S, 4, 4, 14, nsc, 2)
            nv_all = ul.d_nv.cpu().numpy().reshape(-1, 4)
            xs = x.cpu().numpy()
            nsamp = xs.size // 2 // (S * 4)
            print(f"== snr {snr} seed {seed}: compact vs per-symbol LLRs {stats(res['compact'], res['per_symbol'])}",
                  flush=True)
            for s in range(S):
                off = ul.llr_offsets[s]
                n = sum(sg.cw_length for sg in cell.segs)
                A = res["per_symbol"][off:off + n]
                # B: the reference chain on the same samples.
                B = np.zeros(n, np.int8)
                o1, o2 = ctypes.c_longlong(), ctypes.c_longlong()
                samp = np.ascontiguousarray(xs[2 * s * 4 * nsamp: 2 * (s + 1) * 4 * nsamp])
                rb0 = np.zeros(1, np.int32)
                nrb = np.array([273], np.int32)
                lib.ref_ul_slot_timed_at(1, rb0.ctypes.data_as(P_), nrb.ctypes.data_as(P_), qm,
                                         ctypes.c_uint(cell.dmrs_mask), 1, cell.slot_index(s),
                                         samp.ctypes.data_as(P_), B.ctypes.data_as(P_), ctypes.byref(o1),
                                         ctypes.byref(o2))
                # C: the reference OFDM demodulator alone.
                rgrid = ref.ofdm_demodulate(samp.view(np.complex64).reshape(4, nsamp), 1, 273, 4096, False, 1.0 / 64,
                                            3.5e9, cell.slot_index(s) % 2)
                g = grid_all[s]
                gw = g.view(np.uint32)[..., 0]
                rw = rgrid.view(np.uint32)[..., 0]
                gdiff = int(np.sum(gw != rw))
                # D: reference estimator + demodulator on the GPU grid.
                ccfg = dict(slot=cell.slot_index(s), scrambling_id=500, n_scid=0, dmrs_type2=0,
                            scaling=slotlib.DMRS_BETA, dmrs_symbol_mask=cell.dmrs_mask, start_symbol=0, nof_symbols=14,
                            rb_start=0, nof_rb=273, nof_rx_ports=4)
                rce, rnv, rrsrp, _, _, rcfo = ref.pusch_chest(ccfg, g, 273, fd=2, td=0, compensate_cfo=True)
                dcfg = dict(rnti=0x4601, n_id=500, qm=qm, nof_layers=1, nof_rx_ports=4, start_symbol=0,
                            nof_symbols=14, dmrs_symbol_mask=cell.dmrs_mask, dmrs_type2=0,
                            nof_cdm_groups_without_data=2, rb_start=0, nof_rb=273)
                D = ref.pusch_demodulate(dcfg, g, rce, rnv, 273)
                # E: reference demodulator on the GPU's grid, estimates and noise variances.
                gce = ce_all[s, 0]  # layer 0: (ports, 14, nsc, 2)
                E = ref.pusch_demodulate(dcfg, g, gce, nv_all[s], 273)
                cw = ce_all[s, 0].view(np.uint32)[..., 0]
                rcw = rce.view(np.uint32)[..., 0]
                ce_diff = int(np.sum(cw != rcw))
                ce_err = np.abs(bf16_to_complex(gce) - bf16_to_complex(rce)).max() / np.sqrt(
                    np.mean(np.abs(bf16_to_complex(rce)) ** 2))
                print(f"  slot {s}: A(gpu) vs B(ref chain) {stats(A, B)}", flush=True)
                print(f"     grid words differing (C) {gdiff} of {gw.size}; estimate words differing {ce_diff} of "
                      f"{cw.size} (max err/rms {ce_err:.2e}); nv gpu {nv_all[s]} ref {rnv}", flush=True)
                print(f"     A vs D (ref est+demod on gpu grid) {stats(A, D)}", flush=True)
                print(f"     A vs E (ref demod on gpu grid+est+nv) {stats(A, E)}", flush=True)
                print(f"     E vs D (estimates only) {stats(E, D)}", flush=True)
                d = np.abs(A.astype(np.int16) - B.astype(np.int16))
                for i in np.nonzero(d > 1)[0][:12]:
                    r, bit = divmod(int(i), qm)
                    l, sc = data_syms[r // nsc], r % nsc
                    yg = bf16_to_complex(g[:, l, sc])
                    yr = bf16_to_complex(rgrid[:, l, sc])
                    hg = bf16_to_complex(gce[:, l, sc])
                    hr = bf16_to_complex(rce[:, l, sc])
                    print(f"     llr {i}: sym {l} sc {sc} bit {bit}: gpu {A[i]} ref {B[i]} D {D[i]} E {E[i]}; "
                          f"y gpu {np.round(yg, 5)} ref {np.round(yr, 5)}; h gpu {np.round(hg, 5)} ref "
                          f"{np.round(hr, 5)}", flush=True)


if __name__ == "__main__":
    main()
