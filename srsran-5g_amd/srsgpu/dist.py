"""Multi-GPU sharding of the slot batch and the gather of decoded transport blocks to the FAPI rank.

North star (BASELINE.json): "code blocks / UE allocations within a slot batch shard naturally across the 8 GPUs of
one node with an RCCL-over-xGMI gather of decoded TBs back to the FAPI adaptor". One process per GPU:

* every rank runs the whole PDSCH/PUSCH channel-coding pipeline on its own share of the batch (cells, or the UE
  allocations of a slot) - codeblocks never cross GPUs, so the data path has no collective;
* the only exchange is the uplink result: the decoded transport blocks and their CRC flags of every rank go to the
  rank that hosts the FAPI adaptor (the reference's `fapi_adaptor` PUSCH results path, one point of delivery to the
  MAC), with one RCCL gather per batch (torch.distributed "nccl" = RCCL on ROCm; "gloo" on CPU for the tests).

The downlink needs no exchange: each rank's encoded codewords go to its own radio units.
"""
from __future__ import annotations

from typing import List, Optional, Sequence

import torch
import torch.distributed as dist


def shard_range(n_items: int, world: int, rank: int) -> range:
    """Contiguous, balanced share [begin, end) of n_items for `rank` (sizes differ by at most one)."""
    if world <= 0 or not 0 <= rank < world:
        raise ValueError("invalid world/rank")
    base, extra = divmod(n_items, world)
    begin = rank * base + min(rank, extra)
    return range(begin, begin + base + (1 if rank < extra else 0))


def shard_ues(ues: Sequence, world: int, rank: int) -> List:
    """The UE allocations of a slot batch that `rank` processes (UE granularity keeps every TB on one GPU)."""
    return [ues[i] for i in shard_range(len(ues), world, rank)]


class TbGather:
    """Gathers every rank's decoded-TB bytes and CRC flags into `root`'s buffers.

    Ranks may hold different amounts (a UE shard's TB sizes differ from another's): the sizes are exchanged once at
    construction (one all_gather), every rank sends a buffer padded to the largest, and on the root `tbs[r]` /
    `crc_ok[r]` are views of rank r's real bytes. `gather` is one collective pair per batch on the current stream; the
    buffers are allocated once (per plan). `assemble()` concatenates the ranks' results in rank order, which is the
    UE order of the slot for contiguous `shard_ues` shares.
    """

    def __init__(self, tb_bytes: int, nof_tbs: int, device: torch.device, root: int = 0,
                 group: Optional[dist.ProcessGroup] = None):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.root = root
        self.group = group
        self.tb_bytes = int(tb_bytes)
        self.nof_tbs = int(nof_tbs)
        mine = torch.tensor([self.tb_bytes, self.nof_tbs], dtype=torch.int64, device=device)
        sizes = [torch.zeros(2, dtype=torch.int64, device=device) for _ in range(self.world)]
        dist.all_gather(sizes, mine, group=group)
        self.sizes = [(int(x[0]), int(x[1])) for x in sizes]
        self.max_bytes = max(b for b, _ in self.sizes)
        self.max_tbs = max(n for _, n in self.sizes)
        self._send_tbs = torch.zeros(self.max_bytes, dtype=torch.uint8, device=device)
        self._send_ok = torch.zeros(self.max_tbs, dtype=torch.uint8, device=device)
        if self.rank == root:
            self._recv_tbs = [torch.empty(self.max_bytes, dtype=torch.uint8, device=device) for _ in range(self.world)]
            self._recv_ok = [torch.empty(self.max_tbs, dtype=torch.uint8, device=device) for _ in range(self.world)]
            self.tbs = [t[:b] for t, (b, _) in zip(self._recv_tbs, self.sizes)]
            self.crc_ok = [t[:n] for t, (_, n) in zip(self._recv_ok, self.sizes)]
        else:
            self._recv_tbs = self._recv_ok = None
            self.tbs = None
            self.crc_ok = None

    def gather(self, d_tbs: torch.Tensor, d_crc_ok: torch.Tensor) -> None:
        if d_tbs.numel() != self.tb_bytes or d_crc_ok.numel() != self.nof_tbs:
            raise ValueError("TB buffer sizes differ from the ones the gather was planned for")
        self._send_tbs[: self.tb_bytes].copy_(d_tbs)
        self._send_ok[: self.nof_tbs].copy_(d_crc_ok)
        dist.gather(self._send_tbs, self._recv_tbs, dst=self.root, group=self.group)
        dist.gather(self._send_ok, self._recv_ok, dst=self.root, group=self.group)

    def assemble(self):
        """Root only: (all TB bytes, all CRC flags) in rank order."""
        if self.rank != self.root:
            raise ValueError("only the root holds the gathered results")
        return torch.cat(self.tbs), torch.cat(self.crc_ok)
