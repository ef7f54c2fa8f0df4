"""Frequency allocations and reserved resource-element patterns of the PDSCH / PUSCH transmissions (host side).

The GPU plans take a CRB mask (one byte per grid CRB) and reserved RE patterns (srsgpu_alloc_ext, include/srsgpu_phy.h);
this module builds them the way the reference does:

- ``vrb_to_crb_mask``: rb_allocation::get_crb_mask (lib/phy/upper/rb_allocation.cpp:76) over the non-interleaved and
  interleaved VRB-to-PRB mappings of TS 38.211 7.3.1.6 (lib/ran/resource_allocation/vrb_to_prb.cpp:81, :94, :243),
  with the interleaver configurations of include/srsran/ran/resource_allocation/vrb_to_prb.h:80-:189;
- ``ReservedPattern``: re_pattern (include/srsran/phy/support/re_pattern.h): CRBs x PRB subcarriers x symbols;
- ``count_data_res``: the data REs of an allocation after the DM-RS and reserved patterns are excluded
  (pdsch_modulator_impl.cpp:58-:104, resource_grid_mapper_impl.cpp:299-:303).
"""
from __future__ import annotations

from dataclasses import dataclass, field
from typing import Optional, Sequence

import numpy as np


@dataclass
class VrbToPrbConfig:
    """vrb_to_prb::configuration (vrb_to_prb.h:37); nof_bundles == 0 means non-interleaved."""
    nof_bundles: int = 0
    coreset_start: int = 0
    nof_rbs: int = 0
    first_bundle_size: int = 0
    other_bundle_size: int = 0
    last_bundle_size: int = 0

    @property
    def interleaved(self) -> bool:
        return self.nof_bundles != 0


def _ceil_div(a: int, b: int) -> int:
    return -(-a // b)


def non_interleaved_common_ss(coreset_start: int) -> VrbToPrbConfig:
    """TS 38.211 7.3.1.6 case 1 (vrb_to_prb.h:80): VRB n -> PRB n + N_start^CORESET."""
    return VrbToPrbConfig(coreset_start=coreset_start)


def non_interleaved_other() -> VrbToPrbConfig:
    """TS 38.211 7.3.1.6 case 2 (vrb_to_prb.h:92): VRB n -> PRB n."""
    return VrbToPrbConfig()


def interleaved_coreset0(coreset_start: int, bwp_init_size: int) -> VrbToPrbConfig:
    """TS 38.211 7.3.1.6 case 3 (vrb_to_prb.h:111): bundle size 2 over CORESET0."""
    L = 2
    return VrbToPrbConfig(_ceil_div(bwp_init_size, L), coreset_start, bwp_init_size, L, L,
                          bwp_init_size % L if bwp_init_size % L else L)


def interleaved_common_ss(coreset_start: int, bwp_start: int, bwp_init_size: int) -> VrbToPrbConfig:
    """TS 38.211 7.3.1.6 case 4 (vrb_to_prb.h:146)."""
    L = 2
    s = (bwp_start + coreset_start) % L
    e = (bwp_init_size + bwp_start + coreset_start) % L
    return VrbToPrbConfig(_ceil_div(bwp_init_size + s, L), coreset_start, bwp_init_size, L - s, L, e if e else L)


def interleaved_other(bwp_start: int, bwp_size: int, bundle_size: int) -> VrbToPrbConfig:
    """TS 38.211 7.3.1.6 case 5 (vrb_to_prb.h:177): bundle size L_i in {2, 4}."""
    L = int(bundle_size)
    if L not in (2, 4):
        raise ValueError(f"invalid RB bundle size {L} (2 or 4)")
    e = (bwp_start + bwp_size) % L
    return VrbToPrbConfig(_ceil_div(bwp_size + bwp_start % L, L), 0, bwp_size, L - bwp_start % L, L, e if e else L)


def interleaved_vrb_to_prb(cfg: VrbToPrbConfig) -> np.ndarray:
    """PRB of every VRB of an interleaved mapping: first and last bundles in place, bundle j (0 < j < N - 1) of the
    R = 2 row, C = N / 2 column block interleaver to PRB bundle f(j) = r C + c for j = c R + r
    (vrb_to_prb.cpp:94)."""
    N, R = cfg.nof_bundles, 2
    C = N // R
    out = np.zeros(cfg.nof_rbs, np.int64)
    f, o = cfg.first_bundle_size, cfg.other_bundle_size
    out[:f] = cfg.coreset_start + np.arange(f)
    last = cfg.last_bundle_size
    out[cfg.nof_rbs - last:] = cfg.coreset_start + (N - 2) * o + f + np.arange(last)
    for c in range(C):
        for r in range(R):
            j = c * R + r
            if j == 0 or j > N - 2:
                continue
            fj = r * C + c
            out[(j - 1) * o + f:(j - 1) * o + f + o] = cfg.coreset_start + (fj - 1) * o + f + np.arange(o)
    return out


def vrb_to_crb_mask(vrb_mask: Sequence[int], bwp_start: int, bwp_size: int, grid_nof_prb: int,
                    vrb_to_prb: Optional[VrbToPrbConfig] = None) -> np.ndarray:
    """rb_allocation::get_crb_mask: one uint8 per grid CRB, set for the CRBs the allocated VRBs map to."""
    vrbs = np.flatnonzero(np.asarray(vrb_mask))
    cfg = vrb_to_prb or VrbToPrbConfig()
    if cfg.interleaved:
        if len(vrb_mask) > cfg.nof_rbs or cfg.coreset_start + cfg.nof_rbs > bwp_size:
            raise ValueError("VRB bitmap larger than the interleaver or interleaver larger than the BWP")
        prbs = interleaved_vrb_to_prb(cfg)[vrbs]
    else:
        if cfg.coreset_start + len(vrb_mask) > bwp_size:
            raise ValueError("VRB bitmap does not fit the BWP")
        prbs = cfg.coreset_start + vrbs
    if bwp_start + bwp_size > grid_nof_prb:
        raise ValueError("BWP outside the grid")
    out = np.zeros(grid_nof_prb, np.uint8)
    out[bwp_start + prbs] = 1
    return out


@dataclass
class ReservedPattern:
    """re_pattern (re_pattern.h): the PRB subcarriers of re_mask (bit k = subcarrier k) in every CRB of crb_mask
    (None = all CRBs) and every OFDM symbol of symbol_mask (bit l = symbol l)."""
    re_mask: int
    symbol_mask: int
    crb_mask: Optional[np.ndarray] = None

    @staticmethod
    def from_range(rb_begin: int, rb_end: int, rb_stride: int, re_mask: int, symbol_mask: int, grid_nof_prb: int):
        """re_pattern(rb_begin, rb_end, rb_stride, re_mask, symbols) (re_pattern.h)."""
        m = np.zeros(grid_nof_prb, np.uint8)
        m[rb_begin:rb_end:rb_stride] = 1
        return ReservedPattern(re_mask, symbol_mask, m)


def dmrs_prb_mask(dmrs_type: int, nof_cdm_groups_without_data: int) -> int:
    """DM-RS subcarriers of a PRB (dmrs_mapping.h get_dmrs_prb_mask): type 1 CDM group g on 2k + g, type 2 on
    6k + 2g + {0, 1}."""
    m = 0
    for k in range(12):
        g = (k % 6) // 2 if dmrs_type == 2 else k % 2
        if g < nof_cdm_groups_without_data:
            m |= 1 << k
    return m


def count_data_res(grid_nof_prb: int, crb_mask: np.ndarray, start_symbol: int, nof_symbols: int,
                   dmrs_symbol_mask: int, dmrs_type: int, nof_cdm_groups_without_data: int, bwp_start: int,
                   bwp_size: int, reserved: Sequence[ReservedPattern] = ()) -> int:
    """Data REs: the allocated CRBs' subcarriers over the allocated symbols, minus the BWP's DM-RS pattern on DM-RS
    symbols and the reserved patterns."""
    crbs = np.asarray(crb_mask, np.uint8) != 0
    dm = dmrs_prb_mask(dmrs_type, nof_cdm_groups_without_data)
    in_bwp = np.zeros(grid_nof_prb, bool)
    in_bwp[bwp_start:bwp_start + bwp_size] = True
    n = 0
    for l in range(start_symbol, start_symbol + nof_symbols):
        excl = np.zeros(grid_nof_prb, np.int64)
        if (dmrs_symbol_mask >> l) & 1:
            excl[in_bwp] |= dm
        for r in reserved:
            if (r.symbol_mask >> l) & 1:
                sel = np.ones(grid_nof_prb, bool) if r.crb_mask is None else np.asarray(r.crb_mask) != 0
                excl[sel] |= r.re_mask & 0xFFF
        free = 12 - np.array([bin(int(x)).count("1") for x in excl])
        n += int(free[crbs].sum())
    return n
