"""UL-SCH demultiplexer (UCI on PUSCH) test configurations: random allocations, DM-RS patterns and HARQ-ACK / CSI Part 1
/ CSI Part 2 sizes that fit the allocation (every UCI field completes, as the reference asserts at the end of the
codeword). TEST INFRASTRUCTURE ONLY."""
import numpy as np

import ulsch_demux_oracle as U


def _fits(cfg, csi2, csi2_first_symbol=0):
    lq = cfg["qm"] * cfg["nof_layers"]
    plan = U.symbol_plan(cfg, csi2, csi2_first_symbol)
    got = {k: sum(len(s[k]) for _, _, s in plan) * lq for k in ("harq", "csi1", "csi2")}
    return (got["harq"] == cfg["nof_enc_harq_ack_bits"] and got["csi1"] == cfg["nof_enc_csi_part1_bits"]
            and got["csi2"] == csi2)


def random_config(rng, max_prb=20, allow_first_empty=False, csi2_after_csi1=False):
    """Returns (cfg, nof_csi_part2_bits, nof_enc_csi_part2_bits, c_init). csi2_after_csi1: CSI Part 2 (when present)
    placed from the symbol that completes CSI Part 1 on, the PUSCH processor's timing; the returned configurations
    then have CSI Part 1 and CSI Part 2 whenever possible."""
    while True:
        qm = int(rng.choice([2, 4, 6, 8]))
        L = int(rng.choice([1, 2]))
        lq = qm * L
        nprb = int(rng.integers(1, max_prb + 1))
        start = int(rng.integers(0, 3))
        nsym = int(rng.integers(8, 15 - start))
        first = start + int(rng.integers(0, 3))
        mask = 1 << first
        if rng.random() < 0.3:
            mask |= 1 << (first + 1)
        if rng.random() < 0.6 and first + 7 < start + nsym:
            mask |= 1 << (first + 7)
        t2 = int(rng.random() < 0.3)
        cdm = int(rng.integers(1, 4 if t2 else 3))
        cap = 12 * nprb * (nsym - 4)  # rough UCI capacity in REs
        hb = int(rng.choice([0, 1, 2, 5, 11, 20]))
        he = lq * int(rng.integers(1, max(2, cap // 8))) if hb else 0
        rvd = 0
        if 0 < hb <= 2:
            rvd = he + lq * int(rng.integers(0, 3))
        elif hb == 0 and rng.random() < 0.3:
            rvd = lq * int(rng.integers(1, 6))
        cb = int(rng.choice([1, 2, 7, 30] if csi2_after_csi1 else [0, 0, 1, 2, 7, 30]))
        ce = lq * int(rng.integers(1, max(2, cap // 8))) if cb else 0
        c2b = int(rng.choice([1, 2, 40] if csi2_after_csi1 else [0, 0, 1, 2, 40])) if cb else 0
        c2e = lq * int(rng.integers(1, max(2, cap // 10))) if c2b else 0
        cfg = dict(qm=qm, nof_layers=L, nof_prb=nprb, start_symbol=start, nof_symbols=nsym, dmrs_symbol_mask=mask,
                   dmrs_type2=t2, nof_cdm_groups_without_data=cdm, nof_harq_ack_rvd=rvd, nof_harq_ack_bits=hb,
                   nof_enc_harq_ack_bits=he, nof_csi_part1_bits=cb, nof_enc_csi_part1_bits=ce)
        # The reference loops forever when the first allocated symbol carries no data (a DM-RS symbol with every RE
        # taken by CDM groups, type 2 with three groups): ulsch_demultiplex_impl::on_new_block only skips empty
        # symbols after completing one. Such allocations are left out of the reference comparison.
        first_empty = (mask >> start) & 1 and (4 if t2 else 6) * cdm == 12
        first_csi2 = (U.csi1_end_symbol(cfg) or 0) if csi2_after_csi1 else 0
        if (allow_first_empty or not first_empty) and _fits(cfg, c2e, first_csi2):
            return cfg, c2b, c2e, int(rng.integers(0, 1 << 31))


def nof_llrs(cfg):
    lq = cfg["qm"] * cfg["nof_layers"]
    return sum(M for _, M, _ in U.symbol_plan(cfg)) * lq
