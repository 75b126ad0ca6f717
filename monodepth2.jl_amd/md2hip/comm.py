"""RCCL data parallelism through the library's own C-ABI communicator (md2_comm_*; include/md2.h).

One process per GPU.  Rank 0 creates the 128-byte RCCL id (``unique_id()``) and ships it to the
other ranks by any channel (here: a torch.distributed *gloo* broadcast, i.e. host control plane
only -- gradients never pass through torch); ``Comm(rank, nranks, id, device)`` joins.  A train step
is ``train_step_dp`` (md2_model_train_step_dp): forward_loss, then per backward segment the RCCL
sum of its gradient bucket on the communicator's stream, overlapped with the rest of the backward
(SURVEY.md 8(e)), then ONE ADAM (1/nranks) + weight re-pack after the last bucket.  With
MD2_SEG_UPDATE=1 each bucket's ADAM + re-pack instead runs on the executor's update stream right
after its all-reduce (opt-in: measured 2% slower at N=1).  ``backward_allreduce`` is the all-reduce half
alone (md2_model_backward_allreduce)."""
from __future__ import annotations

import ctypes as C

from ._lib import check, declare, lib, ptr, stream_of

P = C.c_void_p
ID_BYTES = 128

declare("md2_comm_get_unique_id", C.c_int, [C.c_char_p])
declare("md2_comm_init", C.c_int, [C.c_int, C.c_int, C.c_char_p, C.c_int, C.POINTER(C.c_void_p)])
declare("md2_comm_destroy", C.c_int, [P])
declare("md2_comm_rank", C.c_int, [P, C.POINTER(C.c_int), C.POINTER(C.c_int)])
declare("md2_comm_stats", C.c_int, [P, C.POINTER(C.c_longlong), C.POINTER(C.c_longlong)])
declare("md2_comm_allreduce_sum", C.c_int, [P, P, C.c_longlong, P])
declare("md2_model_backward_allreduce", C.c_int, [P, P, P])
declare("md2_model_train_step_dp", C.c_int, [P, P, P, P, P, P, C.c_float, C.c_float, C.c_float, C.c_float,
                                             C.c_int, P, P])


def unique_id() -> bytes:
    buf = C.create_string_buffer(ID_BYTES)
    check(lib().md2_comm_get_unique_id(buf), "md2_comm_get_unique_id")
    return buf.raw


def broadcast_id(rank: int, group=None) -> bytes:
    """Rank 0's RCCL id to every rank over an initialised (gloo) torch.distributed group."""
    import torch.distributed as dist
    obj = [unique_id() if rank == 0 else None]
    dist.broadcast_object_list(obj, src=0, group=group)
    return obj[0]


class Comm:
    """``md2_comm``: one RCCL rank on ``device`` with its own comm stream."""

    def __init__(self, rank: int, nranks: int, uid: bytes, device: int = 0):
        if len(uid) != ID_BYTES:
            raise ValueError("RCCL unique id must be 128 bytes")
        h = C.c_void_p()
        check(lib().md2_comm_init(rank, nranks, C.create_string_buffer(uid, ID_BYTES), device, C.byref(h)),
              "md2_comm_init")
        self.handle, self.rank, self.nranks = h, rank, nranks

    def close(self):
        if self.handle:
            lib().md2_comm_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def query(self):
        """(rank, nranks) as the RCCL communicator itself reports them (md2_comm_rank)."""
        r, n = C.c_int(), C.c_int()
        check(lib().md2_comm_rank(self.handle, C.byref(r), C.byref(n)), "md2_comm_rank")
        return r.value, n.value

    def stats(self):
        """(all-reduce calls, payload bytes) enqueued through this communicator so far."""
        calls, nbytes = C.c_longlong(), C.c_longlong()
        check(lib().md2_comm_stats(self.handle, C.byref(calls), C.byref(nbytes)), "md2_comm_stats")
        return calls.value, nbytes.value

    def allreduce_sum(self, t):
        """In-place sum over ranks of a float32 CUDA tensor, ordered on the current stream."""
        check(lib().md2_comm_allreduce_sum(self.handle, ptr(t), t.numel(), stream_of(t.device)),
              "md2_comm_allreduce_sum")
        return t

    @property
    def grad_scale(self) -> float:
        return 1.0 / self.nranks


def backward_allreduce(executor, comm: Comm | None):
    """All backward segments with their overlapped bucket all-reduce (comm None: plain backward)."""
    check(lib().md2_model_backward_allreduce(executor.handle, comm.handle if comm else None,
                                             stream_of(executor.model.device)),
          "md2_model_backward_allreduce")


def train_step_dp(executor, model, opt, x, comm: Comm | None, loss=None):
    """forward_loss -> backward with bucketed RCCL all-reduce -> ADAM(grad_scale = 1/nranks)."""
    out = executor.forward_loss(x, None, loss=loss)
    backward_allreduce(executor, comm)
    opt.update(model, grad_scale=comm.grad_scale if comm else 1.0)
    return out
