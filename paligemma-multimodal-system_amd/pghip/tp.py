"""Tensor-parallel communicator for the Gemma decoder.

One process per GPU.  The only data-path collective is an in-place SUM all-reduce of
fp32 partial sums — after o_proj, after down_proj, and for the vocabulary-parallel
lm_head (each rank writes its slot of a zeroed buffer, so the SUM is an all-gather) —
issued on the current HIP stream through torch.distributed: backend "nccl" is RCCL
over xGMI on the MI355X node (capturable into the decode hipGraph), "gloo" is the CPU
transport used by the world-size-2 tests.  The reference has no parallelism at all
(single device, modeling_gemma.py / inference.py); this replaces nothing there.
"""
from __future__ import annotations

import torch


class TPComm:
    def __init__(self, group=None):
        import torch.distributed as dist
        if not dist.is_initialized():
            raise RuntimeError("TPComm: torch.distributed is not initialised")
        self._dist = dist
        self.group = group
        self.rank = dist.get_rank(group)
        self.world = dist.get_world_size(group)
        self.backend = dist.get_backend(group)
        self.capturable = self.backend == "nccl"      # RCCL collectives can live inside a hipGraph

    def all_reduce(self, t: torch.Tensor):
        self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group)


class SoloComm:
    """World of one: no collectives."""
    rank, world, backend, capturable = 0, 1, "none", True

    def all_reduce(self, t: torch.Tensor):
        return None
