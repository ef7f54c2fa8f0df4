"""Host SCH logic (TBS, base graph, segmentation) against the reference segmenter (ldpc_segmenter_tx_impl) run through
the reference build; plus TBS sanity values."""
import numpy as np
import pytest

from oracle_lib import Reference, have_ref
from srsgpu import sch


def test_tbs_known_values():
    # 273 PRB, 4 layers, MCS 27 (table 2), 1 DM-RS symbol: the srsRAN maximum-TBS case (sch_constants.h:43).
    g = sch.UeGrant(273, 4, 8, 948)
    assert g.tbs == 1277992
    assert sch.UeGrant(4, 4, 8, 948).tbs == 18432
    assert sch.tbs_calculate(1, 12, 12, 0, 2, 120, 1) == 24  # N_info = 30.9 -> N_info' = 24


@pytest.mark.skipif(not have_ref(), reason="reference build absent")
@pytest.mark.parametrize("case", [
    (4, 4, 8, 948), (5, 4, 8, 948), (273, 4, 8, 948), (51, 1, 6, 772), (10, 2, 4, 434), (2, 1, 2, 120),
    (1, 1, 2, 193), (106, 2, 8, 682.5), (24, 3, 6, 517)])
def test_segmentation_matches_reference(case):
    n_prb, layers, qm, r = case
    g = sch.UeGrant(n_prb, layers, qm, r)
    seg = g.segmentation()
    ref = Reference()
    rng = np.random.default_rng(n_prb)
    tb = rng.integers(0, 256, seg.tbs // 8).astype(np.uint8)
    _, meta = ref.pdsch_encode(seg.base_graph, 0, qm, layers, 0, g.nof_ch_symbols, tb)
    assert meta.shape[0] == seg.nof_segments
    for cb, m in zip(seg.codeblocks, meta):
        assert (cb.lifting_size, cb.nof_filler_bits, cb.rm_length, cb.nof_info_bits) == tuple(int(x) for x in m)
