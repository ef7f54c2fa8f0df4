"""TEST INFRASTRUCTURE ONLY -- numpy restatement ("oracle") of the srsRAN UL-SCH demultiplexer (UCI on PUSCH, TS 38.212
section 6.2.7): per OFDM symbol, the RE sets of the reserved HARQ-ACK REs, HARQ-ACK, CSI Part 1, CSI Part 2 and UL-SCH
data, and the routing of the demodulated, descrambled LLRs to the four decoder buffers, with the placeholder handling of
1- and 2-bit UCI. Only tests/ may use it, as the checker. Pinned against the reference's own ulsch_demultiplex_impl
(oracle/ref/ref_ulsch_demux.cpp) by tests/test_oracle_vs_reference.py.

Reference files (under /root/reference/lib/phy/upper/channel_processors/pusch/):
  ulsch_demultiplex_impl.cpp:29   l1: first symbol without DM-RS after the first DM-RS symbol; l1_csi: first symbol
                                  without DM-RS (:45)
  ulsch_demultiplex_impl.cpp:68   re_set_select: every d-th available RE, m_re_count of them
  ulsch_demultiplex_impl.cpp:316  configure_current_ofdm_symbol: steps 1 (reserved HARQ-ACK), 2 (HARQ-ACK > 2 bits),
                                  3 (CSI Part 1), 3bis (CSI Part 2), 5 (HARQ-ACK <= 2 bits on the reserved REs)
  ulsch_demultiplex_impl.cpp:91   on_uci_placeholder_1bit: per modulation symbol, bit 1 takes the scrambling of bit 0
                                  ("y"), bits >= 2 are unscrambled ("x")
  ulsch_demultiplex_impl.cpp:131  on_uci_placeholder_2bit: bits >= 2 unscrambled
  ulsch_demultiplex_impl.cpp:455  demux_current_ofdm_symbol: HARQ-ACK (<= 2 bits: the REs are zeroed for the UL-SCH),
                                  CSI Part 1, CSI Part 2, then the UL-SCH REs in order
"""
import numpy as np

import pusch_demod_oracle as D


def _select(avail, d, count):
    """re_set_select: from the available RE indices (ascending) every d-th one, count of them."""
    return [int(i) for i in avail[::d][:count]]


def symbol_plan(cfg, csi2_enc_bits=0, csi2_first_symbol=0):
    """Per allocated OFDM symbol: (symbol, M REs, dict of RE index lists: rvd, harq, csi1, csi2, ulsch).

    cfg: qm, nof_layers, nof_prb, start_symbol, nof_symbols, dmrs_symbol_mask, dmrs_type2, nof_cdm_groups_without_data,
    nof_harq_ack_rvd, nof_harq_ack_bits, nof_enc_harq_ack_bits, nof_csi_part1_bits, nof_enc_csi_part1_bits
    (ulsch_demultiplex::configuration); csi2_enc_bits: G^CSI-2, placed from symbol csi2_first_symbol on (where
    set_csi_part2 is called, ulsch_demultiplex_impl.cpp:241; 0: before the first symbol)."""
    lq = cfg["qm"] * cfg["nof_layers"]
    mask = cfg["dmrs_symbol_mask"]
    dm = [(mask >> l) & 1 for l in range(14)]
    first_dmrs = dm.index(1)
    l1 = next(l for l in range(first_dmrs, 14) if not dm[l])
    l1_csi = dm.index(0)
    per_rb_dmrs = (4 if cfg["dmrs_type2"] else 6) * cfg["nof_cdm_groups_without_data"]
    m_rvd = m_harq = m_csi1 = m_csi2 = 0
    out = []
    for l in range(cfg["start_symbol"], cfg["start_symbol"] + cfg["nof_symbols"]):
        M = (12 - per_rb_dmrs) * cfg["nof_prb"] if dm[l] else 12 * cfg["nof_prb"]
        ulsch = np.ones(M, bool)
        uci = np.full(M, not dm[l])
        sets = dict(rvd=[], harq=[], csi1=[], csi2=[])
        M_uci = int(uci.sum())
        # Step 1: reserved REs for HARQ-ACK.
        rem_rvd = (cfg["nof_harq_ack_rvd"] - m_rvd) // lq
        if l >= l1 and M_uci > 0 and rem_rvd > 0:
            d, n = (M_uci // rem_rvd, rem_rvd) if rem_rvd < M_uci else (1, M_uci)
            sets["rvd"] = _select(np.flatnonzero(ulsch), d, n)
            m_rvd += n * lq
        # Step 2: HARQ-ACK of more than two bits.
        rem_harq = (cfg["nof_enc_harq_ack_bits"] - m_harq) // lq
        if l >= l1 and M_uci > 0 and cfg["nof_harq_ack_bits"] > 2 and rem_harq > 0:
            d, n = (M_uci // rem_harq, rem_harq) if rem_harq < M_uci else (1, M_uci)
            sets["harq"] = _select(np.flatnonzero(uci), d, n)
            ulsch[sets["harq"]] = False
            uci[sets["harq"]] = False
            M_uci = int(uci.sum())
            m_harq += n * lq
        # Step 3: CSI Part 1 outside the reserved REs.
        rem_csi1 = (cfg["nof_enc_csi_part1_bits"] - m_csi1) // lq
        M_r = len(sets["rvd"])
        if l >= l1_csi and M_uci - M_r > 0 and rem_csi1 > 0:
            avail = np.ones(M, bool)
            avail[sets["rvd"]] = False
            avail &= uci
            d, n = ((M_uci - M_r) // rem_csi1, rem_csi1) if rem_csi1 < M_uci - M_r else (1, M_uci - M_r)
            sets["csi1"] = _select(np.flatnonzero(avail), d, n)
            ulsch[sets["csi1"]] = False
            uci[sets["csi1"]] = False
            m_csi1 += n * lq
        # Step 3bis: CSI Part 2.
        M_uci = int(uci.sum())
        rem_csi2 = (csi2_enc_bits - m_csi2) // lq
        if l >= l1_csi and l >= csi2_first_symbol and M_uci > 0 and rem_csi2 > 0:
            d, n = (M_uci // rem_csi2, rem_csi2) if rem_csi2 < M_uci else (1, M_uci)
            sets["csi2"] = _select(np.flatnonzero(uci), d, n)
            ulsch[sets["csi2"]] = False
            uci[sets["csi2"]] = False
            m_csi2 += n * lq
        # Step 5: HARQ-ACK of up to two bits on the reserved REs (which stay in the UL-SCH set).
        if M_r > 0 and cfg["nof_harq_ack_bits"] <= 2 and rem_harq > 0:
            d, n = (M_r // rem_harq, rem_harq) if rem_harq < M_r else (1, M_r)
            sets["harq"] = _select(np.array(sets["rvd"]), d, n)
            m_harq += n * lq
        sets["ulsch"] = [int(i) for i in np.flatnonzero(ulsch)]
        out.append((l, M, sets))
    return out


def _placeholder(re_llr, seq_bits, qm, nbits):
    """on_uci_placeholder_1bit / _2bit over one RE's LLRs (layers x qm); seq_bits: the scrambling bits of those LLRs."""
    v = re_llr.astype(np.int16).copy()
    for s in range(0, v.size, qm):
        if nbits == 1:
            if seq_bits[s] ^ seq_bits[s + 1]:
                v[s + 1] = -v[s + 1]
        for i in range(2, qm):
            if seq_bits[s + i]:
                v[s + i] = -v[s + i]
    return v.astype(np.int8)


def csi1_end_symbol(cfg):
    """The OFDM symbol whose demultiplexing completes CSI Part 1 (where the reference's PUSCH processor decodes it and
    calls set_csi_part2, pusch_processor_impl.cpp:72-100); None without CSI Part 1."""
    last = None
    for l, _M, sets in symbol_plan(cfg):
        if sets["csi1"]:
            last = l
    return last


def demultiplex(cfg, llrs, c_init, csi2_bits=0, csi2_enc_bits=0, csi2_first_symbol=0):
    """Routes the descrambled codeword LLRs (int8, demodulation order) of one transmission. Returns dict of int8 arrays:
    sch, harq, csi1, csi2 (the LLRs each decoder buffer receives, in order). csi2_first_symbol: see symbol_plan."""
    qm, lq = cfg["qm"], cfg["qm"] * cfg["nof_layers"]
    seq = D.gold_sequence(c_init, llrs.size)
    out = dict(sch=[], harq=[], csi1=[], csi2=[])
    nbits = dict(harq=cfg["nof_harq_ack_bits"], csi1=cfg["nof_csi_part1_bits"], csi2=csi2_bits)
    pos = 0
    for _l, M, sets in symbol_plan(cfg, csi2_enc_bits, csi2_first_symbol):
        data = llrs[pos: pos + M * lq].astype(np.int8).copy().reshape(M, lq)
        sb = seq[pos: pos + M * lq].reshape(M, lq)
        for kind in ("harq", "csi1", "csi2"):
            for r in sets[kind]:
                if nbits[kind] in (1, 2) and qm > 1:
                    out[kind].append(_placeholder(data[r], sb[r], qm, nbits[kind]))
                    if kind == "harq":
                        data[r] = 0
                else:
                    out[kind].append(data[r].copy())
        for r in sets["ulsch"]:
            out["sch"].append(data[r])
        pos += M * lq
    return {k: (np.concatenate(v) if v else np.zeros(0, np.int8)) for k, v in out.items()}
