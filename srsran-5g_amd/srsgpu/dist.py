"""Multi-GPU sharding of the slot batch and the gather of decoded transport blocks to the FAPI rank.

North star (BASELINE.json): "code blocks / UE allocations within a slot batch shard naturally across the 8 GPUs of
one node with an RCCL-over-xGMI gather of decoded TBs back to the FAPI adaptor". One process per GPU:

* sharding by cell (weak scaling, the bench's default): every rank runs the whole pipeline, OFDM included, on its
  own cells' slots - codeblocks never cross GPUs, so the data path has no collective; the only exchange is the
  uplink result: the decoded transport blocks and their CRC flags of every rank go to the rank that hosts the FAPI
  adaptor (the reference's `fapi_adaptor` PUSCH results path, one point of delivery to the MAC), with one RCCL gather
  per batch (`TbGather`; torch.distributed "nccl" = RCCL on ROCm; "gloo" on CPU for the tests);
* sharding the UEs of one cell (strong scaling): a cell's samples enter and leave on one rank, so the resource grid
  is exchanged as well (`GridExchange`): the root's demodulated UL grid is scattered by subcarrier band to the ranks
  that own the UEs there, and the ranks' DL grid bands are gathered into the root's grid before its OFDM modulation;
  the decoded TBs go to the FAPI rank through `TbGather` as above;
* sharding the codeblocks of a slot (strong scaling where one UE owns the cell: configs[4]'s test-mode UE carries
  ~140 codeblocks per slot, which UE sharding cannot split): the FAPI rank runs the front end and holds the codeword
  LLRs, every rank decodes a contiguous range of the slot's codeblocks into its own HARQ buffers and the messages come
  back for the TB assembly (`CodeblockShard`).
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
    construction (one all_gather), every rank sends one buffer - its TB bytes padded to the largest rank's, then its
    CRC flags padded the same way - so a batch costs one collective (the host issues a collective per step at a few
    thousand steps per second), and on the root `tbs[r]` / `crc_ok[r]` are views of rank r's real bytes. `gather` runs
    on the current stream; the buffers are allocated once (per plan). `assemble()` concatenates the ranks' results in
    rank order, which is the UE order of the slot for contiguous `shard_ues` shares.
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
        self._send = torch.zeros(self.max_bytes + self.max_tbs, dtype=torch.uint8, device=device)
        if self.rank == root:
            self._recv = [torch.empty(self.max_bytes + self.max_tbs, dtype=torch.uint8, device=device)
                          for _ in range(self.world)]
            self.tbs = [t[:b] for t, (b, _) in zip(self._recv, self.sizes)]
            self.crc_ok = [t[self.max_bytes: self.max_bytes + n] for t, (_, n) in zip(self._recv, self.sizes)]
        else:
            self._recv = None
            self.tbs = None
            self.crc_ok = None

    def gather(self, d_tbs: torch.Tensor, d_crc_ok: torch.Tensor) -> None:
        if d_tbs.numel() != self.tb_bytes or d_crc_ok.numel() != self.nof_tbs:
            raise ValueError("TB buffer sizes differ from the ones the gather was planned for")
        self._send[: self.tb_bytes].copy_(d_tbs)
        self._send[self.max_bytes: self.max_bytes + self.nof_tbs].copy_(d_crc_ok)
        dist.gather(self._send, self._recv, dst=self.root, group=self.group)

    def assemble(self):
        """Root only: (all TB bytes, all CRC flags) in rank order."""
        if self.rank != self.root:
            raise ValueError("only the root holds the gathered results")
        return torch.cat(self.tbs), torch.cat(self.crc_ok)


def ue_subcarrier_ranges(ues: Sequence, world: int) -> List[tuple]:
    """Subcarrier range [begin, end) of every rank's UE share (contiguous shard_ues shares of contiguous PRB
    allocations starting at PRB 0): the grid columns a rank's UEs occupy."""
    if world <= 0:
        raise ValueError("invalid world")
    out, rb = [], 0
    for r in range(world):
        n = sum(ues[i].n_prb for i in shard_range(len(ues), world, r))
        out.append((12 * rb, 12 * (rb + n)))
        rb += n
    return out


class GridExchange:
    """The resource-grid exchange of a cell whose UEs are split across ranks (strong scaling, `--shard ues`).

    The cell's radio samples enter and leave on one rank, the root (it hosts the cell's radio unit link): the root runs
    the OFDM demodulation / modulation of the whole cell, the other ranks only the upper PHY of their UEs. Uplink: the
    root's demodulated grid is cut into the ranks' subcarrier ranges and scattered (`scatter`); each rank writes its
    range into its own full-width grid, where its UEs' estimator / demodulator plans read it. Downlink: every rank maps
    its UEs into its grid and the ranges are gathered into the root's grid (`gather`) before the OFDM modulation.

    The grid is [rows][nsc] int32 (rows = slots x ports x symbols, bf16 pairs), a rank's range is a column band, so a
    transfer packs it into a dense send buffer (one strided device copy) padded to the widest band (RCCL's scatter /
    gather move equal chunks). Per step each non-root rank moves rows x width x 4 bytes in each direction; the root
    sends / receives the sum over the others. Buffers are allocated once; all copies and collectives run on the current
    stream (graph-capturable with RCCL).
    """

    def __init__(self, rows: int, nsc: int, sc_ranges: Sequence[tuple], device: torch.device, root: int = 0,
                 group: Optional[dist.ProcessGroup] = None):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if len(sc_ranges) != self.world:
            raise ValueError("one subcarrier range per rank")
        for b, e in sc_ranges:
            if not 0 <= b <= e <= nsc:
                raise ValueError(f"subcarrier range [{b}, {e}) outside the grid's {nsc}")
        self.rows, self.nsc, self.root, self.group = int(rows), int(nsc), root, group
        self.ranges = [(int(b), int(e)) for b, e in sc_ranges]
        self.width = max(e - b for b, e in self.ranges)
        self._mine = torch.zeros(self.rows, self.width, dtype=torch.int32, device=device)
        self._all = ([torch.zeros(self.rows, self.width, dtype=torch.int32, device=device) for _ in range(self.world)]
                     if self.rank == root else None)

    @property
    def bytes_per_rank(self) -> List[int]:
        """Grid bytes of every rank's band (what one scatter or gather moves to / from that rank)."""
        return [self.rows * (e - b) * 4 for b, e in self.ranges]

    def _grid2d(self, d_grid: torch.Tensor) -> torch.Tensor:
        if d_grid.dtype != torch.int32 or d_grid.numel() != self.rows * self.nsc:
            raise ValueError(f"grid of {d_grid.numel()} {d_grid.dtype} words, the exchange was planned for "
                             f"{self.rows} x {self.nsc} int32")
        return d_grid.view(self.rows, self.nsc)

    def scatter(self, d_grid: torch.Tensor) -> None:
        """Uplink: the root's bands of `d_grid` go to their ranks' `d_grid` (same columns)."""
        g = self._grid2d(d_grid)
        if self.rank == self.root:
            for r, (b, e) in enumerate(self.ranges):
                if r != self.root:
                    self._all[r][:, : e - b].copy_(g[:, b:e])
        dist.scatter(self._mine, self._all, src=self.root, group=self.group)
        if self.rank != self.root:
            b, e = self.ranges[self.rank]
            g[:, b:e].copy_(self._mine[:, : e - b])

    def gather(self, d_grid: torch.Tensor) -> None:
        """Downlink: every rank's band of its `d_grid` goes into the root's `d_grid` (same columns)."""
        g = self._grid2d(d_grid)
        b, e = self.ranges[self.rank]
        if self.rank != self.root:
            self._mine[:, : e - b].copy_(g[:, b:e])
        dist.gather(self._mine, self._all, dst=self.root, group=self.group)
        if self.rank == self.root:
            for r, (b, e) in enumerate(self.ranges):
                if r != self.root:
                    g[:, b:e].copy_(self._all[r][:, : e - b])


CB_MSG_STRIDE = 1056  # SRSGPU_CB_MSG_STRIDE: bytes per codeblock message slot


class CodeblockShard:
    """Codeblock-level sharding of a slot's PUSCH decoding across ranks.

    `cbs` lists the slot's codeblocks in order (every TB's, concatenated) as (llr_offset, rm_length) in the root's
    codeword LLR buffer. Ownership: without `keys`, rank r owns the contiguous codeblock range
    `shard_range(len(cbs), world, r)` (one contiguous LLR span each) - valid for slots of new transmissions only, since a
    retransmitted TB's codeblocks move with the slot's composition. With `keys` (one stable HARQ key per codeblock, e.g.
    the rx buffer pool's absolute codeblock identifier, rx_buffer.h:65), codeblock i belongs to rank keys[i] mod world in
    every slot, so a retransmission is decoded by the rank whose HARQ buffer holds the earlier transmissions' soft bits
    (its LLRs are packed per rank for the scatter).

    Per slot: `scatter_llrs` hands every rank its codeblocks' LLRs (one scatter; the root keeps its own); each rank
    rate-dematches and decodes its codeblocks into its own HARQ buffers (a srsgpu_pusch_cb_plan over `local_cbs`, LLR
    offsets relative to its buffer: the HARQ memory is sharded as well); `gather` brings the messages (CB_MSG_STRIDE bytes
    each) and CRC flags into the root's slot-wide buffers (one gather), where srsgpu_pusch_decoder_plan_assemble joins
    them into TBs and checks the TB CRCs (pusch_decoder_impl.cpp:386); `return_flags` scatters the root's final flags
    back, so a TB CRC mismatch clears the owners' codeblock flags exactly as the reference resets them for the
    retransmission (:423). Buffers and the per-rank index tensors are allocated once; copies and collectives run on the
    current stream, one indexed copy per rank on the root.

    With `keys`, a rank's local codeblock positions change from slot to slot, so its CRC flags - the HARQ context that
    makes the reference skip a codeblock already decoded in an earlier transmission (pusch_decoder_impl.cpp:208,
    rx_buffer.h `get_codeblocks_crc`) - belong to the key, not the position: `return_flags(..., harq_flags=t)` also
    stores them into `t[key]` (a per-rank tensor indexed by HARQ key, like the HBM HARQ arena), and
    `local_flags(t)` reads this slot's local codeblocks' flags back in local order.
    """

    def __init__(self, cbs: Sequence[tuple], device: torch.device, root: int = 0,
                 group: Optional[dist.ProcessGroup] = None, keys: Optional[Sequence[int]] = None):
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.root, self.group = root, group
        self.cbs = [(int(o), int(e)) for o, e in cbs]
        for (o, e), (o2, _) in zip(self.cbs, self.cbs[1:]):
            if o2 < o + e:
                raise ValueError("codeblock LLR ranges must be in order and disjoint")
        if keys is None:
            #: codeblock indices (slot order) each rank decodes
            self.members = [list(shard_range(len(self.cbs), self.world, r)) for r in range(self.world)]
        else:
            if len(keys) != len(self.cbs):
                raise ValueError("one HARQ key per codeblock")
            self.members = [[i for i, k in enumerate(keys) if int(k) % self.world == r] for r in range(self.world)]
        #: per rank: (first LLR, count) pieces of the root's buffer it receives, contiguous pieces merged
        self.pieces = []
        for mem in self.members:
            pcs = []
            for i in mem:
                o, e = self.cbs[i]
                if pcs and pcs[-1][0] + pcs[-1][1] == o:
                    pcs[-1] = (pcs[-1][0], pcs[-1][1] + e)
                else:
                    pcs.append((o, e))
            self.pieces.append(pcs)
        self.spans = [sum(n for _, n in pcs) for pcs in self.pieces]
        self.max_span = max(1, max(self.spans))
        self.max_cbs = max(1, max(len(m) for m in self.members))
        #: (llr_offset relative to this rank's buffer, rm_length) of the codeblocks this rank decodes
        self.local_cbs = []
        pos = 0
        for i in self.members[self.rank]:
            self.local_cbs.append((pos, self.cbs[i][1]))
            pos += self.cbs[i][1]
        self.keys = None if keys is None else [int(k) for k in keys]
        #: this rank's codeblocks' HARQ keys in local order (keyed flags), on the device
        self._local_keys = (torch.tensor([self.keys[i] for i in self.members[self.rank]], dtype=torch.long,
                                         device=device) if self.keys is not None else None)
        #: root: per rank, the slot positions of its codeblocks (indexed copies instead of one copy per codeblock)
        self._idx = ([torch.tensor(m, dtype=torch.long, device=device) for m in self.members] if self.rank == root
                     else None)
        self.llrs = torch.zeros(self.max_span, dtype=torch.int8, device=device)
        self._res = torch.zeros(self.max_cbs * (CB_MSG_STRIDE + 1), dtype=torch.uint8, device=device)
        self._flags = torch.zeros(self.max_cbs, dtype=torch.uint8, device=device)
        if self.rank == root:
            self._llr_all = [torch.zeros(self.max_span, dtype=torch.int8, device=device) for _ in range(self.world)]
            self._res_all = [torch.zeros_like(self._res) for _ in range(self.world)]
            self._flags_all = [torch.zeros(self.max_cbs, dtype=torch.uint8, device=device) for _ in range(self.world)]
        else:
            self._llr_all = self._res_all = self._flags_all = None

    @property
    def ranges(self) -> List[List[int]]:
        """Codeblock indices each rank decodes (slot order)."""
        return self.members

    @property
    def llr_bytes_per_rank(self) -> List[int]:
        return list(self.spans)

    def scatter_llrs(self, d_llrs: Optional[torch.Tensor]) -> torch.Tensor:
        """Root: `d_llrs` is the slot's codeword LLR buffer (other ranks pass None). Returns this rank's LLRs (its
        codeblocks' rate-matched LLRs, packed in slot order)."""
        if self.rank == self.root:
            for r, pcs in enumerate(self.pieces):
                pos = 0
                for b, n in pcs:
                    self._llr_all[r][pos:pos + n].copy_(d_llrs[b:b + n])
                    pos += n
        dist.scatter(self.llrs, self._llr_all, src=self.root, group=self.group)
        return self.llrs[: self.spans[self.rank]]

    def gather(self, d_msgs: torch.Tensor, d_flags: torch.Tensor, d_all_msgs: Optional[torch.Tensor],
               d_all_flags: Optional[torch.Tensor]) -> None:
        """This rank's messages (len(local_cbs) x CB_MSG_STRIDE bytes) and flags into the root's slot-wide buffers
        (codeblock i at i x CB_MSG_STRIDE; the other ranks pass None for the root's buffers)."""
        n = len(self.local_cbs)
        if d_msgs.numel() < n * CB_MSG_STRIDE or d_flags.numel() < n:
            raise ValueError("message / flag buffers smaller than this rank's codeblocks")
        self._res[: n * CB_MSG_STRIDE].copy_(d_msgs[: n * CB_MSG_STRIDE])
        self._res[self.max_cbs * CB_MSG_STRIDE: self.max_cbs * CB_MSG_STRIDE + n].copy_(d_flags[:n])
        dist.gather(self._res, self._res_all, dst=self.root, group=self.group)
        if self.rank == self.root:
            S = CB_MSG_STRIDE
            total = len(self.cbs)
            msgs2d = d_all_msgs[: total * S].view(total, S)
            for r, mem in enumerate(self.members):
                if not mem:
                    continue
                k = len(mem)
                src = self._res_all[r]
                msgs2d.index_copy_(0, self._idx[r], src[: k * S].view(k, S))
                d_all_flags.index_copy_(0, self._idx[r], src[self.max_cbs * S: self.max_cbs * S + k])

    def return_flags(self, d_all_flags: Optional[torch.Tensor], d_flags: torch.Tensor,
                     harq_flags: Optional[torch.Tensor] = None) -> None:
        """The root's codeblock flags after the TB stage back to their owners' `d_flags` (local order); with
        `harq_flags` (keyed sharding) also into harq_flags[key], the HARQ context that follows the codeblock."""
        if self.rank == self.root:
            for r, mem in enumerate(self.members):
                if mem:
                    self._flags_all[r][: len(mem)].copy_(d_all_flags.index_select(0, self._idx[r]))
        dist.scatter(self._flags, self._flags_all, src=self.root, group=self.group)
        n = len(self.local_cbs)
        d_flags[:n].copy_(self._flags[:n])
        if harq_flags is not None:
            if self._local_keys is None:
                raise ValueError("keyed flags need the shard's HARQ keys")
            if n:
                harq_flags.index_copy_(0, self._local_keys, self._flags[:n].to(harq_flags.dtype))

    def local_flags(self, harq_flags: torch.Tensor) -> torch.Tensor:
        """This slot's local codeblocks' CRC flags from the keyed HARQ context (local order): what this rank's decoder
        reads to skip the codeblocks an earlier transmission already decoded."""
        if self._local_keys is None:
            raise ValueError("keyed flags need the shard's HARQ keys")
        return harq_flags.index_select(0, self._local_keys)
