"""Tensor-parallel communicator for the Gemma decoder.

One process per GPU.  The data-path collectives are
  * an in-place SUM all-reduce of fp32 partial sums after o_proj and after down_proj (row-parallel linears);
  * an all-gather in rank order: the vocabulary-parallel lm_head logits (top-p / full logits) and, when the
    batch covers the ranks, the SigLIP features of the images each rank encoded (data-parallel vision).
They are issued on the current HIP stream, either through torch.distributed (TPComm: backend "nccl" is RCCL over
xGMI on the MI355X node, capturable into the decode hipGraph; "gloo" is the CPU transport of the world-size-2
tests) or as peer-store kernels over xGMI (XgmiComm, csrc/allreduce.hip): the one-shot pg_allreduce_xgmi /
pg_allgather_xgmi for decode-size messages, the reduce-scatter + all-gather pg_allreduce_xgmi_rs for the prefill's
megabyte row chunks.  all_reduce_async lets the prefill overlap a chunk's all-reduce
with the next chunk's GEMM (the returned handle's wait() orders the current stream after the collective).  The
reference has no parallelism at all (single device, modeling_gemma.py / inference.py); this replaces nothing there.
"""
from __future__ import annotations

import torch


class CaptureUnsupported(RuntimeError):
    """A collective that cannot run inside a hipGraph capture (PaliGemmaEngine.generate then runs eager steps)."""


class _Done:
    def wait(self):
        return None


class _StreamWork:
    """A collective enqueued on a side stream: wait() makes the current stream wait for it."""

    def __init__(self, event: torch.cuda.Event):
        self.event = event

    def wait(self):
        torch.cuda.current_stream().wait_event(self.event)


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

    def all_reduce_slabs(self, part: torch.Tensor, ns: int) -> int:
        """SUM over the ranks of this rank's ns split-K slabs part[:ns] (contiguous [S][rows][H]), written to part[0]:
        the slabs are summed locally first (ops.slab_sum, fixed slab order), so one slab crosses the links.
        Returns 1, the slab count the next norm must add."""
        if ns > 1:
            from . import ops
            ops.slab_sum(part[:ns], part[0])
        self.all_reduce(part[0])
        return 1

    def all_reduce_async(self, t: torch.Tensor):
        """SUM all-reduce that may run concurrently with later work on the current stream; call .wait() on the
        result before the stream reads t."""
        if self.backend == "gloo":                     # gloo stages device tensors through the host: synchronous
            self.all_reduce(t)
            return _Done()
        return self._dist.all_reduce(t, op=self._dist.ReduceOp.SUM, group=self.group, async_op=True)

    def all_gather(self, out: torch.Tensor, t: torch.Tensor):
        """out (contiguous, world * t.numel() elements) = every rank's t in rank order."""
        self._dist.all_gather_into_tensor(out.view(-1), t.contiguous().view(-1), group=self.group)


class XgmiComm(TPComm):
    """TP communicator whose collectives run as peer-store kernels over xGMI (csrc/allreduce.hip): decode-size
    all-reduces / all-gathers as the one-shot exchange (pg_allreduce_xgmi / pg_allgather_xgmi), all-reduces of more
    than `rs_min` elements -- the prefill's row chunks, up to `rs_cap` -- as a reduce-scatter + all-gather
    (pg_allreduce_xgmi_rs: 2(W-1)/W of the message per rank instead of W-1).  Both sum in rank order,
    so every rank gets the same bits from either.  The process group only exchanges the IPC handles at construction and
    carries what fits neither (non-fp32, unaligned, or too large: counted in `fallbacks`).

    Every rank holds one exchange buffer and one RS buffer; the handles travel through all_gather_object, so this also
    works over gloo (ranks sharing one device in the tests).  Because the kernels keep their epoch counters on the
    device, the collectives are graph-capturable whatever the backend, so `capturable` is True.  A collective that does
    not fit (`fits(numel)` False) raises CaptureUnsupported inside a capture; PaliGemmaEngine.generate and bench.py then
    fall back to eager decode steps.

    The RS grid (`rs_wg` workgroups) is 256 with one rank per device; ranks that share a device split the device's
    256 between them (a workgroup spins until the same workgroup of every peer has stored, so the ranks' grids must
    all be resident at once, csrc/allreduce.hip)."""

    def __init__(self, group=None, cap: int = 1 << 22, rs_cap: int = 1 << 23, rs_min: int = 1 << 18,
                 rs_wg: int | None = None):
        super().__init__(group)
        import ctypes as C
        import socket
        from . import _lib
        if cap % 4 or rs_cap % 4 or rs_cap < 0:
            raise ValueError("XgmiComm: cap and rs_cap must be multiples of 4 (rs_cap 0 disables the RS form)")
        if self.world > 8:
            raise ValueError("XgmiComm: at most 8 ranks (one node)")
        self._C, self._lib, self.cap, self.rs_cap, self.rs_min = C, _lib, cap, rs_cap, rs_min
        self._opened = []
        self._own = self._own_rs = None
        self._peers = self._map(self._alloc("pg_xgmi_buffer_bytes", cap))
        # ranks per device: which ranks share this process's device (host name + PCI bus id)
        dev = torch.cuda.current_device()
        props = torch.cuda.get_device_properties(dev)
        key = (socket.gethostname(), getattr(props, "pci_bus_id", None), getattr(props, "pci_device_id", None),
               str(getattr(props, "uuid", dev)))
        keys = [None] * self.world
        self._dist.all_gather_object(keys, key, group=self.group)
        self.ranks_per_device = max(keys.count(k) for k in keys)
        self.rs_wg = rs_wg if rs_wg is not None else max(8, 256 // self.ranks_per_device)
        if not 1 <= self.rs_wg <= 256:
            raise ValueError("XgmiComm: rs_wg must be in 1..256")
        self._peers_rs = self._map(self._alloc("pg_xgmi_rs_buffer_bytes", rs_cap), rs=True) if rs_cap else None
        self.epochs = torch.zeros(64, dtype=torch.int32, device="cuda")
        self.epochs_rs = torch.zeros(256, dtype=torch.int32, device="cuda")
        self.err_diag = torch.zeros(8, dtype=torch.int32, device="cuda")   # see include/pghip.h: err[0..6]
        self.err = self.err_diag[:1]
        self._side = None
        self.fallbacks = 0                            # collectives carried by the process group instead (too large)
        self.rs_calls = 0                             # all-reduces that ran as reduce-scatter + all-gather
        self._dist.barrier(group=self.group)          # every rank mapped every buffer before first use
        self.capturable = True

    def _alloc(self, size_fn: str, cap: int):
        C = self._C
        nbytes = C.c_long()
        self._lib.call(size_fn, self.world, cap, C.byref(nbytes))
        own = C.c_void_p()
        self._lib.call("pg_xgmi_alloc", nbytes.value, C.byref(own))
        return own.value

    def _map(self, own, rs=False):
        """Exchange this rank's buffer handle with every rank; map the peers' buffers; peers[r] in this process."""
        C = self._C
        if rs:
            self._own_rs = own
        else:
            self._own = own
        h = C.create_string_buffer(64)
        self._lib.call("pg_xgmi_ipc_handle", own, h)
        handles = [None] * self.world
        self._dist.all_gather_object(handles, h.raw, group=self.group)
        peers = (C.c_void_p * self.world)()
        for r, hr in enumerate(handles):
            if r == self.rank:
                peers[r] = own
                continue
            m = C.c_void_p()
            self._lib.call("pg_xgmi_ipc_open", C.create_string_buffer(hr, 64), C.byref(m))
            peers[r] = m.value
            self._opened.append(m.value)
        return peers

    def fits(self, numel: int) -> bool:
        return 0 < numel and numel % 4 == 0 and (numel <= self.cap or self._rs_fits(numel))

    def _rs_fits(self, numel: int) -> bool:
        return self._peers_rs is not None and self.rs_min < numel <= self.rs_cap and numel % 4 == 0

    def _dev_f32(self, t: torch.Tensor) -> bool:
        return t.is_cuda and t.dtype == torch.float32 and t.is_contiguous() and t.data_ptr() % 16 == 0

    def _ok(self, t: torch.Tensor) -> bool:
        return self._dev_f32(t) and self.fits(t.numel())

    def _refuse_in_capture(self, what: str, t: torch.Tensor):
        if torch.cuda.is_current_stream_capturing():
            raise CaptureUnsupported(f"XgmiComm: {what} of {t.numel()} x {t.dtype} does not fit the exchange "
                                     f"buffers (cap {self.cap}, rs_cap {self.rs_cap} fp32) inside a graph capture")

    def _rs(self, t: torch.Tensor, nslab: int = 1, stride: int = 0):
        self.rs_calls += 1
        self._lib.call("pg_allreduce_xgmi_rs", t.data_ptr(), t.numel(), nslab, stride, self.rank, self.world,
                       self._peers_rs, self.rs_cap, self.rs_wg, self.epochs_rs.data_ptr(), self.err_diag.data_ptr(),
                       torch.cuda.current_stream().cuda_stream)

    def all_reduce(self, t: torch.Tensor):
        if self._dev_f32(t) and self._rs_fits(t.numel()):
            self._rs(t)
        elif self._dev_f32(t) and self.fits(t.numel()):
            self._lib.call("pg_allreduce_xgmi", t.data_ptr(), t.numel(), self.rank, self.world, self._peers,
                           self.cap, self.epochs.data_ptr(), self.err_diag.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
        else:
            self._refuse_in_capture("all-reduce", t)
            self.fallbacks += 1
            super().all_reduce(t)

    def all_reduce_slabs(self, part: torch.Tensor, ns: int) -> int:
        """As TPComm.all_reduce_slabs, with the slab sum done inside the exchange kernel (pg_allreduce_xgmi_slabs /
        pg_allreduce_xgmi_rs: the same slab order, one launch)."""
        t = part[0]
        if ns > 1 and self._dev_f32(t) and part.is_contiguous():
            if self._rs_fits(t.numel()):
                self._rs(t, ns, part.stride(0))
                return 1
            if t.numel() <= self.cap:
                self._lib.call("pg_allreduce_xgmi_slabs", t.data_ptr(), t.numel(), ns, part.stride(0), self.rank,
                               self.world, self._peers, self.cap, self.epochs.data_ptr(), self.err_diag.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
                return 1
        return super().all_reduce_slabs(part, ns)

    def all_reduce_async(self, t: torch.Tensor):
        if not self._ok(t):
            if self.backend != "gloo":                # (gloo runs it through self.all_reduce, which counts it)
                self.fallbacks += 1
            return super().all_reduce_async(t)
        # the exchange on a side stream that first waits for everything enqueued so far on the current one
        if self._side is None:
            self._side = torch.cuda.Stream()
        self._side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(self._side):
            self.all_reduce(t)
            ev = torch.cuda.Event()
            ev.record(self._side)
        return _StreamWork(ev)

    def all_gather(self, out: torch.Tensor, t: torch.Tensor):
        t = t.contiguous()
        n = t.numel()
        if (self._dev_f32(t) and 0 < n <= self.cap and n % 4 == 0 and out.is_contiguous()
                and out.numel() == self.world * n and out.data_ptr() % 16 == 0):
            self._lib.call("pg_allgather_xgmi", t.data_ptr(), n, out.data_ptr(), self.rank, self.world,
                           self._peers, self.cap, self.epochs.data_ptr(), self.err_diag.data_ptr(),
                           torch.cuda.current_stream().cuda_stream)
        elif (t.is_cuda and t.dtype == torch.float32 and n > self.cap and n % 4 == 0 and out.is_contiguous()
              and out.numel() == self.world * n and t.data_ptr() % 16 == 0 and not torch.cuda.is_current_stream_capturing()):
            # larger than the exchange (the SigLIP features of several images per rank): pieces of at most `cap`
            # elements, each gathered into a [world][piece] staging tensor and copied to its rank-strided place
            piece = self.cap
            stage = torch.empty(self.world, piece, dtype=torch.float32, device=t.device)
            ov = out.view(self.world, n)
            for k0 in range(0, n, piece):
                k1 = min(n, k0 + piece)
                st = stage[:, : k1 - k0]
                if k1 - k0 < piece:
                    st = stage.view(-1)[: self.world * (k1 - k0)].view(self.world, k1 - k0)
                self._lib.call("pg_allgather_xgmi", t.data_ptr() + 4 * k0, k1 - k0, st.data_ptr(), self.rank,
                               self.world, self._peers, self.cap, self.epochs.data_ptr(), self.err_diag.data_ptr(),
                               torch.cuda.current_stream().cuda_stream)
                ov[:, k0:k1].copy_(st)
        else:
            self._refuse_in_capture("all-gather", t)
            self.fallbacks += 1
            super().all_gather(out, t)

    def diagnostics(self) -> dict:
        """The first timed-out exchange of this rank (include/pghip.h err[0..6]), or {} if none."""
        d = self.err_diag.tolist()
        if not d[0]:
            return {}
        kinds = {1: "one-shot", 2: "reduce-scatter", 3: "rs all-gather"}
        return {"kind": kinds.get(d[1], d[1]), "workgroup": d[2], "peer": d[3], "expected_epoch": d[4],
                "seen_flag": d[5], "rank": d[6]}

    def check(self):
        """Raise if any exchange timed out waiting for a peer (results since then are invalid)."""
        d = self.diagnostics()
        if d:
            raise RuntimeError(f"pg_allreduce_xgmi: a peer did not arrive within the timeout: {d}")

    def close(self):
        if self._own is None:
            return
        torch.cuda.synchronize()
        self._dist.barrier(group=self.group)          # no peer still writes into our buffers
        for m in self._opened:
            self._lib.call("pg_xgmi_ipc_close", m)
        self._dist.barrier(group=self.group)
        self._lib.call("pg_xgmi_free", self._own)
        if self._own_rs is not None:
            self._lib.call("pg_xgmi_free", self._own_rs)
        self._own, self._own_rs, self._opened = None, None, []


class SoloComm:
    """World of one: no collectives."""
    rank, world, backend, capturable = 0, 1, "none", True

    def all_reduce(self, t: torch.Tensor):
        return None

    def all_reduce_async(self, t: torch.Tensor):
        return _Done()

    def all_gather(self, out: torch.Tensor, t: torch.Tensor):
        out.view(-1).copy_(t.reshape(-1))
