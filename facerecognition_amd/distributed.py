"""Data-parallel embed + sharded gallery match across ranks.

One process per GPU.  Rank r embeds its own batch of faces; the gallery is row-sharded (rank r holds
global rows [lo_r, hi_r), searched with ``index_base = lo_r``).  The one real exchange step:

  1. all-gather the L2-normalized embeddings  [B, D] per rank → [world*B, D] on every rank
  2. every rank: local top-k of ALL gathered probes against its shard (global indices)
  3. all-gather the candidates [world*B, k] (score, idx) per rank → [world, world*B, k]
  4. every rank: deterministic merge per probe, (score desc, global index asc)

Because the ordering is total and every candidate list is itself exact, the merged top-k equals the
single-device top-k over the whole gallery bit for bit (tests/test_distributed.py checks this with
world_size 2 on gloo).  On GPUs the collectives are RCCL over xGMI (backend "nccl") and steps 2/4 are
``fr_match_topk`` / ``fr_topk_merge``; on CPU (tests) the same protocol runs with numpy callables.

The reference has no multi-process path; this is the scale-out the north star asks for.
"""
from __future__ import annotations

from typing import Callable, Optional, Tuple

import torch


def shard_range(rows: int, rank: int, world: int) -> Tuple[int, int]:
    """Contiguous, balanced row range of `rank` (sizes differ by at most one row)."""
    return rank * rows // world, (rank + 1) * rows // world


def _all_gather(out: torch.Tensor, inp: torch.Tensor, group=None) -> None:
    import torch.distributed as dist
    if dist.get_backend(group) == "nccl":
        dist.all_gather_into_tensor(out, inp.contiguous(), group=group)
    else:  # gloo (CPU tests, or several ranks sharing one GPU in the -m gpu test): list form,
        # staged through host memory when the tensors live on the device
        world = dist.get_world_size(group)
        host = out if not out.is_cuda else torch.empty(out.shape, dtype=out.dtype)
        parts = list(host.view(world, *inp.shape).unbind(0))
        dist.all_gather(parts, inp.contiguous().cpu(), group=group)
        if host is not out:
            out.copy_(host)


def native_merge(cand_s: torch.Tensor, cand_i: torch.Tensor, k: int) -> Tuple[torch.Tensor, torch.Tensor]:
    """fr_topk_merge on the device: cand_* [P, n_lists, k] → [P, k]."""
    from . import _native as N
    P, n_lists = int(cand_s.shape[0]), int(cand_s.shape[1])
    s = torch.empty((P, k), dtype=torch.float32, device=cand_s.device)
    i = torch.empty((P, k), dtype=torch.int32, device=cand_s.device)
    N.check(N.lib().fr_topk_merge(N.ptr(cand_s), N.ptr(cand_i), P, n_lists, k, N.ptr(s), N.ptr(i),
                                  N.stream_ptr(cand_s.device)), "fr_topk_merge")
    return s, i


def native_merge_ranks(xchg: torch.Tensor, k: int, out_s: torch.Tensor, out_i: torch.Tensor) -> None:
    """fr_topk_merge_ranks on the device: the all-gathered exchange block xchg [world, 2, P, k] (int32 words:
    rank r's scores as f32 bits, then its global indices) → out_s / out_i [P, k]."""
    from . import _native as N
    W, P = int(xchg.shape[0]), int(xchg.shape[2])
    N.check(N.lib().fr_topk_merge_ranks(N.ptr(xchg), W, P, k, N.ptr(out_s), N.ptr(out_i), N.stream_ptr(xchg.device)),
            "fr_topk_merge_ranks")


class ShardedMatcher:
    """Steps 1-4 above with buffers preallocated at construction: no allocation per call.

    local_search(probes [P, D], out_s [P, k] f32, out_i [P, k] int32) writes the shard's top-k (global
      indices) into out_s / out_i -- views into this rank's block of the candidate send buffer -- or
      returns (scores, idx) tensors, which are then copied there; a one-argument callable
      local_search(probes) -> (scores, idx) (the round-3 interface) is accepted too;
    merge(xchg [world, 2, P, k] int32, k, out_s, out_i) merges the all-gathered blocks (default
      native_merge_ranks, fr_topk_merge_ranks).

    The candidate exchange is ONE all-gather: each rank's block is [2][P][k] 4-byte words (its scores,
    then its indices), written in place by the shard search, gathered as is and merged as is.
    search() returns views of buffers owned by the matcher, overwritten by the next call (clone them to keep
    them).

    Short batches (the last, partial batch of a stream; ranks may differ): a rank with B' < batch probes pads its
    block with masked rows (every element PAD_MARK = 2.0, which no L2-normalized embedding holds; a non-degenerate
    probe, so the shard search costs what a real one does), and after the merge every masked row reads (-inf, -1),
    FAISS's "no result".  Rows j*batch + b, b < rank j's count, are rank j's probes; ``valid`` marks them.  The
    masking adds three small device ops per call; ``pad_short=False`` (callers whose batches are always full, such
    as bench.py) skips it.  At world 1 a short batch returns just its B' rows.
    """

    PAD_MARK = 2.0

    def __init__(self, batch: int, dim: int, k: int, local_search: Callable, device: torch.device,
                 merge: Optional[Callable] = None, group=None, always_exchange: bool = False, pad_short: bool = True):
        import torch.distributed as dist
        self.world = dist.get_world_size(group) if dist.is_initialized() else 1
        self.always_exchange = always_exchange  # run steps 1-4 even at world 1 (tests of the collectives)
        self.group, self.k, self.B = group, k, batch
        self.pad_short = pad_short
        self.local_search = local_search
        self.merge = merge or native_merge_ranks
        W, P = self.world, self.world * batch
        self.all_emb = torch.empty((P, dim), dtype=torch.float32, device=device)
        self.send = torch.empty((2, P, k), dtype=torch.int32, device=device)
        self.xchg = torch.empty((W, 2, P, k), dtype=torch.int32, device=device)
        self.out_s = torch.empty((P, k), dtype=torch.float32, device=device)
        self.out_i = torch.empty((P, k), dtype=torch.int32, device=device)
        self._send_s, self._send_i = self.send[0].view(torch.float32), self.send[1]
        self._pad = torch.empty((batch, dim), dtype=torch.float32, device=device) if pad_short else None
        self.valid = torch.ones(P, dtype=torch.bool, device=device)
        import inspect
        # the round-3 interface local_search(probes) -> (scores, idx): ONE positional parameter in all (a defaulted
        # out_s / out_i still makes the three-argument form)
        try:
            params = inspect.signature(local_search).parameters.values()
            n_pos = len([p for p in params if p.kind in (p.POSITIONAL_ONLY, p.POSITIONAL_OR_KEYWORD)])
            var = any(p.kind == p.VAR_POSITIONAL for p in params)
        except (TypeError, ValueError):
            n_pos, var = 3, False
        self._legacy = n_pos <= 1 and not var

    def _local(self, probes, out_s, out_i):
        r = self.local_search(probes) if self._legacy else self.local_search(probes, out_s, out_i)
        if r is not None:
            out_s.copy_(r[0])
            out_i.copy_(r[1])

    def search(self, emb: torch.Tensor):
        """emb: this rank's normalized embeddings [B, D] → top-k of every rank's probes, identical on
        all ranks: (scores [world*B, k], idx [world*B, k]); row j*B + b is rank j's probe b."""
        if self.world == 1 and not self.always_exchange:
            B = int(emb.shape[0])
            if B > self.B:
                raise ValueError(f"ShardedMatcher.search: {B} probes, built for at most {self.B}")
            s, i = self.out_s[:B], self.out_i[:B]
            self._local(emb, s, i)
            return s, i
        B = int(emb.shape[0])
        if B != self.B:
            if B > self.B or not self.pad_short:
                raise ValueError(f"ShardedMatcher.search: {B} probes on a matcher built for {self.B} per rank"
                                 + ("" if B > self.B else " with pad_short=False"))
            self._pad[:B].copy_(emb)
            self._pad[B:].fill_(self.PAD_MARK)
            emb = self._pad
        _all_gather(self.all_emb, emb, self.group)
        self._local(self.all_emb, self._send_s, self._send_i)
        _all_gather(self.xchg.view(-1), self.send.view(-1), self.group)
        self.merge(self.xchg, self.k, self.out_s, self.out_i)
        if self.pad_short:  # masked rows of every rank -> (-inf, -1)
            torch.ne(self.all_emb[:, 0], self.PAD_MARK, out=self.valid)
            inv = ~self.valid[:, None]
            self.out_s.masked_fill_(inv, float("-inf"))
            self.out_i.masked_fill_(inv, -1)
        return self.out_s, self.out_i
