"""TEST INFRASTRUCTURE ONLY — numpy restatement ("oracle") of the srsRAN PDSCH DM-RS processor: sequence generation,
CDM cover codes, per-CDM-group precoding and RE mapping into a bf16 grid, in float32 with the reference's rounding
(each complex product term rounded, layers accumulated in order, bf16 round half to even). Only tests/ may use it, as
the checker. Pinned bit-for-bit against the reference's own dmrs_pdsch_processor_impl built from its sources
(oracle/ref/ref_dmrs_pdsch.cpp) by tests/test_oracle_vs_reference.py and tests/golden/pdsch_dmrs.npz.

Reference files (under /root/reference/lib/phy/):
  upper/signal_processors/dmrs_pdsch_processor_impl.cpp:56   c_init = ((14 n_slot + l + 1)(2 N_ID + 1) 2^17
                                                              + 2 N_ID + n_SCID) mod 2^31, amplitude sqrt(1/2) x
                                                              config amplitude, sequence index from reference_point_k_rb
  upper/signal_processors/dmrs_pdsch_processor_impl.cpp:80   apply_cdm: w_t by l' (previous symbol is DM-RS), w_f on
                                                              odd sequence indices
  upper/signal_processors/dmrs_pdsch_processor_impl.cpp:117  per CDM group: precoding of the group's ports
                                                              (channel_precoder_generic.cpp:27), RE pattern of the group
  upper/signal_processors/dmrs_helper.cpp:36                 patterns and cover codes per port
  upper/signal_processors/dmrs_helper.cpp:64                 sequence over the rb_mask intervals (CRB-mask allocations)
"""
import numpy as np

import pusch_demod_oracle as D

F = np.float32
WF = {0: (1, 1), 1: (1, -1), 2: (1, 1), 3: (1, -1), 4: (1, 1), 5: (1, -1), 6: (1, 1), 7: (1, -1)}
WT = {0: (1, 1), 1: (1, 1), 2: (1, 1), 3: (1, 1), 4: (1, -1), 5: (1, -1), 6: (1, -1), 7: (1, -1)}


def group_pattern(dmrs_type2, g):
    return [2 * g, 2 * g + 1, 2 * g + 6, 2 * g + 7] if dmrs_type2 else [g + 2 * j for j in range(6)]


def to_bf16(v):
    u = np.asarray(v, F).view(np.uint32).astype(np.uint64)
    return ((u + 0x7FFF + ((u >> 16) & 1)) >> 16).astype(np.uint16)


def crb_runs(cfg, grid_nof_prb, crb_mask=None):
    """Allocated CRB intervals [begin, end): the contiguous rb_start / nof_rb allocation, or the runs of crb_mask
    (dmrs_helper.cpp:77 for_each_interval over config_t::rb_mask)."""
    if crb_mask is None:
        return [(cfg["rb_start"], cfg["rb_start"] + cfg["nof_rb"])]
    m = np.asarray(crb_mask, np.uint8)[:grid_nof_prb] != 0
    runs, rb = [], 0
    while rb < m.size:
        if not m[rb]:
            rb += 1
            continue
        e = rb
        while e < m.size and m[e]:
            e += 1
        runs.append((rb, e))
        rb = e
    return runs


def dmrs_map(cfg, weights, grid_nof_prb, crb_mask=None):
    """cfg: slot, scrambling_id, n_scid, dmrs_type2, nof_layers, nof_ports, dmrs_symbol_mask, reference_point_k_rb,
    rb_start, nof_rb, amplitude. weights (P, L) complex64. crb_mask: optional rb_mask (one byte per grid CRB) replacing
    the contiguous allocation. Returns the grid (P, 14, nsc, 2) uint16 (zeros elsewhere)."""
    P, L = cfg["nof_ports"], cfg["nof_layers"]
    t2 = cfg["dmrs_type2"]
    per_rb = 4 if t2 else 6
    nsc = 12 * grid_nof_prb
    grid = np.zeros((P, 14, nsc, 2), np.uint16)
    amp = F(F(np.sqrt(0.5)) * F(cfg["amplitude"]))
    w = np.asarray(weights, np.complex64)
    for l in range(14):
        if not (cfg["dmrs_symbol_mask"] >> l) & 1:
            continue
        lp = 1 if l > 0 and (cfg["dmrs_symbol_mask"] >> (l - 1)) & 1 else 0
        c_init = ((14 * cfg["slot"] + l + 1) * (2 * cfg["scrambling_id"] + 1) * (1 << 17)
                  + 2 * cfg["scrambling_id"] + cfg["n_scid"]) % (1 << 31)
        # dmrs_helper.cpp:64 dmrs_sequence_generate: the sequence of CRB n starts at (n - k_ref) x per_rb; the
        # unallocated CRBs between intervals are skipped, and the CDM w_f index is the position within the
        # concatenated sequence (per_rb is even, so its parity is the position within the PRB).
        rbs = [rb for b, e in crb_runs(cfg, grid_nof_prb, crb_mask) for rb in range(b, e)]
        n = len(rbs) * per_rb
        if n == 0:
            continue
        idx = np.array([(rb - cfg["reference_point_k_rb"]) * per_rb + k for rb in rbs for k in range(per_rb)])
        c = D.gold_sequence(c_init, 2 * (int(idx.max()) + 1))
        re = np.where(c[2 * idx] == 1, -amp, amp).astype(F)
        im = np.where(c[2 * idx + 1] == 1, -amp, amp).astype(F)
        for g in range((L + 1) // 2):
            ports = [q for q in (2 * g, 2 * g + 1) if q < L]
            seqs = []
            for q in ports:
                s = np.ones(n, F) * F(WT[q][lp])
                s[1::2] *= F(WF[q][1])
                seqs.append((re * s, im * s))
            sc = np.array([rb * 12 + k for rb in rbs for k in group_pattern(t2, g)])
            for p in range(P):
                sr = si = None
                for (a, b), q in zip(seqs, ports):
                    wr, wi = F(w[p, q].real), F(w[p, q].imag)
                    pr = (a * wr).astype(F) - (b * wi).astype(F)
                    pi = (a * wi).astype(F) + (b * wr).astype(F)
                    sr = pr if sr is None else (sr + pr).astype(F)
                    si = pi if si is None else (si + pi).astype(F)
                grid[p, l, sc, 0] = to_bf16(sr)
                grid[p, l, sc, 1] = to_bf16(si)
    return grid
