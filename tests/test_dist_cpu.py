"""Multi-process (world size 2, gloo, CPU) tests of the sharding and of the TB gather to the FAPI rank
(srsgpu/dist.py): the same code the bench runs over RCCL on GPUs."""
import os
import socket
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "srsran-5g_amd"))

from srsgpu import dist as sdist  # noqa: E402
from srsgpu import sch  # noqa: E402


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_shard_range_balanced_and_complete():
    for n in (0, 1, 7, 64, 65, 192):
        for world in (1, 2, 3, 8):
            parts = [sdist.shard_range(n, world, r) for r in range(world)]
            flat = [i for p in parts for i in p]
            assert flat == list(range(n))
            sizes = [len(p) for p in parts]
            assert max(sizes) - min(sizes) <= 1
    with pytest.raises(ValueError):
        sdist.shard_range(4, 2, 2)


def test_shard_ues_keeps_tbs_whole():
    ues = sch.slot_100mhz_4x4()
    world = 8
    shards = [sdist.shard_ues(ues, world, r) for r in range(world)]
    assert sum(len(s) for s in shards) == len(ues)
    # Every UE's codeblocks stay on one rank: the per-rank codeblock counts add up to the slot's.
    cbs = [sum(u.segmentation().nof_segments for u in s) for s in shards]
    assert sum(cbs) == sum(u.segmentation().nof_segments for u in ues)


def _worker(rank, world, port, q):
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        dev = torch.device("cpu")
        nof_tbs, tb_bytes = 5, 37
        g = sdist.TbGather(tb_bytes, nof_tbs, dev, root=0)
        results = []
        for step in range(3):
            tbs = torch.full((tb_bytes,), (rank * 16 + step) & 0xFF, dtype=torch.uint8)
            ok = torch.tensor([(rank + step + i) % 2 for i in range(nof_tbs)], dtype=torch.uint8)
            g.gather(tbs, ok)
            if rank == 0:
                results.append(([t.clone().numpy() for t in g.tbs], [c.clone().numpy() for c in g.crc_ok]))
        with pytest.raises(ValueError):
            g.gather(torch.zeros(tb_bytes + 1, dtype=torch.uint8), torch.zeros(nof_tbs, dtype=torch.uint8))
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, results, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def test_tb_gather_world2_gloo():
    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=120)
        assert err is None, err
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert out[1] == []
    assert len(out[0]) == 3
    for step, (tbs, oks) in enumerate(out[0]):
        for r in range(world):
            assert np.all(tbs[r] == ((r * 16 + step) & 0xFF))
            assert list(oks[r]) == [(r + step + i) % 2 for i in range(5)]


def _shard_worker(rank, world, port, q):
    """One rank of a UE-sharded slot: its share of the 64 UEs (shard_ues), the host-side TB sizing of its plans
    (segmentation -> TB bytes / codeblocks, what its PUSCH decoder plan sizes), decoded TBs faked as a function of the
    UE index, and the gather to rank 0."""
    try:
        os.environ["MASTER_ADDR"] = "127.0.0.1"
        os.environ["MASTER_PORT"] = str(port)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ues = sch.slot_100mhz_4x4()
        mine = sdist.shard_range(len(ues), world, rank)
        segs = [ues[i].segmentation() for i in mine]
        tb = [np.full(s.tbs // 8, i & 0xFF, np.uint8) for i, s in zip(mine, segs)]
        ok = np.array([(i * 7) % 3 != 0 for i in mine], np.uint8)
        g = sdist.TbGather(sum(t.size for t in tb), len(tb), torch.device("cpu"), root=0)
        g.gather(torch.from_numpy(np.concatenate(tb)), torch.from_numpy(ok))
        res = None
        if rank == 0:
            all_tbs, all_ok = g.assemble()
            res = (all_tbs.numpy().copy(), all_ok.numpy().copy(), [s for s in g.sizes])
        dist.barrier()
        dist.destroy_process_group()
        q.put((rank, res, None))
    except Exception as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world", [2, 3])
def test_ue_sharded_slot_gather_gloo(world):
    """UE sharding end to end on CPU ranks: uneven shares (64 UEs over 3 ranks) and per-rank TB sizes, gathered to
    rank 0 in the slot's UE order, equal to what the whole slot on one rank would give."""
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=_shard_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    out = {}
    for _ in range(world):
        rank, res, err = q.get(timeout=120)
        assert err is None, err
        out[rank] = res
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    tbs, ok, sizes = out[0]
    ues = sch.slot_100mhz_4x4()
    want_tbs = np.concatenate([np.full(u.segmentation().tbs // 8, i & 0xFF, np.uint8) for i, u in enumerate(ues)])
    want_ok = np.array([(i * 7) % 3 != 0 for i in range(len(ues))], np.uint8)
    assert np.array_equal(tbs, want_tbs) and np.array_equal(ok, want_ok)
    assert len(set(sizes)) > 1 or world == 1  # the ranks' TB sizes differ: the padding path ran
