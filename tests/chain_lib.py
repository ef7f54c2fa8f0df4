"""Oracle compositions of the reference's channel processors (test infrastructure): PDSCH encoding of a transport
block and PUSCH codeblock decoding, built from the oracle stages exactly like the reference composes them."""
import numpy as np

from oracle_lib import BG_K, BG_N_SHORT, CRC16, CRC24A, CRC24B
from srsgpu import sch


def crc_for_tb(seg):
    """pusch_decoder_impl.cpp:34 select_crc: CRC24B when segmented, else the TB CRC (24A / 16)."""
    if seg.nof_segments > 1:
        return CRC24B
    return CRC24A if seg.tbs > 3824 else CRC16


def oracle_pdsch_encode(orc, tb, bg, rv, qm, nof_layers, Nref, nof_ch_symbols):
    """pdsch_encoder_impl::encode (pdsch_encoder_impl.cpp:28): TB CRC, segmentation, CB CRC24B, LDPC, rate match."""
    tbs = tb.size * 8
    seg = sch.segment(tbs, bg, qm, nof_layers, nof_ch_symbols)
    tb_crc = orc.crc_bytes(CRC16 if tbs <= 3824 else CRC24A, tb)
    crc_bits = np.array([(tb_crc >> (seg.nof_tb_crc_bits - 1 - i)) & 1 for i in range(seg.nof_tb_crc_bits)],
                        np.uint8)
    payload = np.concatenate([np.unpackbits(tb), crc_bits])
    cw, msgs = [], []
    K = seg.segment_length
    for cb in seg.codeblocks:
        last = cb.index == seg.nof_segments - 1
        msg = np.zeros(K, np.uint8)
        data = payload[cb.tb_offset: cb.tb_offset + cb.nof_info_bits + (seg.nof_tb_crc_bits if last else 0)]
        msg[:data.size] = data
        used = data.size + (seg.zero_pad if last else 0)
        if seg.cb_crc_bits:
            c = orc.crc_bits(CRC24B, msg[:used])
            msg[used:used + 24] = [(c >> (23 - i)) & 1 for i in range(24)]
        enc = orc.ldpc_encode(bg, seg.lifting_size, msg)
        cw.append(orc.rate_match(bg, seg.lifting_size, rv, qm, Nref, seg.nof_filler_bits, enc, cb.rm_length))
        msgs.append(msg)
    return np.concatenate(cw), seg, msgs


def bits_to_llrs(rng, bits, amp=8.0, noise=0.0):
    llr = (1 - 2 * bits.astype(np.float64)) * amp
    if noise > 0:
        llr = llr + rng.normal(0, noise, llr.size)
    return np.clip(np.round(llr), -120, 120).astype(np.int8)


def oracle_pusch_cb_decode(orc, mode, cb, llr, harq, crc_ok):
    """pusch_decoder_impl.cpp:283 cb task: dematch (always), then decode unless the CB CRC already passed.
    cb: srsgpu.PuschCodeblock. Returns (iterations: int, -1 or 0 when skipped; bits; new harq; new crc flag)."""
    harq = orc.rate_dematch(mode, cb.base_graph, cb.lifting_size, cb.rv, cb.modulation_order, cb.Nref,
                            cb.nof_filler_bits, int(cb.new_data), llr, harq)
    if crc_ok:
        return 0, None, harq, True
    if cb.use_early_stop:
        r, bits = orc.ldpc_decode(mode, cb.base_graph, cb.lifting_size, harq, nof_crc_bits=cb.nof_crc_bits,
                                  nof_filler=cb.nof_filler_bits, crc_poly=cb.crc_poly, max_iter=cb.max_iterations,
                                  scaling=cb.scaling_factor)
    else:
        _, bits = orc.ldpc_decode(mode, cb.base_graph, cb.lifting_size, harq, nof_crc_bits=cb.nof_crc_bits,
                                  nof_filler=cb.nof_filler_bits, crc_poly=-1, max_iter=cb.max_iterations,
                                  scaling=cb.scaling_factor)
        L = BG_K[cb.base_graph] * cb.lifting_size - cb.nof_filler_bits
        r = cb.max_iterations if orc.crc_bits(cb.crc_poly, bits[:L]) == 0 else -1
    return r, bits, harq, r > 0
