"""Native collective transports of the row-sharded tree engine (``h2o_tree_dist`` in
``csrc/tree_kernels.hip``): the whole sharded tree — kernels and collectives — is one native call that enqueues
everything on the compute stream.

* :class:`NativeComm` — an RCCL communicator owned by this process (one process per GPU), driven from C++
  (``csrc/rccl_comm.hip``). Rank 0 draws the unique id and the ``torch.distributed`` process group broadcasts
  it; collectives then go straight over xGMI on the caller's stream, with no Python and no host wait between
  the levels of a tree. The reference's equivalent is the MRTask reduce tree over TCP
  (``h2o-core/src/main/java/water/MRTask.java`` ``reduce2`` / ``water/RPC.java``).
* :class:`HostTransport` — the same native driver with its collectives called back into Python and run by the
  process group's backend on host-staged copies (gloo: CPU tests and several ranks sharing one GPU, which RCCL
  refuses). Slow, but the identical native sequence, layouts and wire dtypes as the RCCL path.

``H2O_NATIVE_COMM=0`` disables the RCCL transport (the host transport is used under any backend).
"""
from __future__ import annotations

import ctypes
import os
import threading

import torch
import torch.distributed as dist

from ..ops import _native as nat
from . import collectives as coll

OP_ALLREDUCE, OP_REDUCE_SCATTER, OP_ALLGATHER = 0, 1, 2
DT_F32, DT_F64, DT_U8 = 0, 1, 2
_DT = {DT_F32: torch.float32, DT_F64: torch.float64, DT_U8: torch.uint8}

_lock = threading.Lock()
_comms: dict = {}


def _rccl_path() -> str:
    return os.path.join(os.path.dirname(torch.__file__), "lib", "librccl.so")


def load_rccl():
    """The HIP library with RCCL resolved (raises if RCCL cannot be loaded)."""
    lib = nat.hip()
    rc = lib.h2o_rccl_load(_rccl_path().encode())
    if rc != 0:
        for alt in ("/opt/rocm/lib/librccl.so.1", "librccl.so.1"):
            rc = lib.h2o_rccl_load(alt.encode())
            if rc == 0:
                break
    if rc != 0:
        raise RuntimeError(f"RCCL could not be loaded (h2o_rccl_load rc={rc})")
    return lib


class NativeComm:
    """An RCCL communicator of ``world`` ranks on the current GPU, created from a broadcast unique id."""

    def __init__(self, world: int, rank: int, uid: bytes):
        self.lib = load_rccl()
        self.world, self.rank = int(world), int(rank)
        self.device = torch.cuda.current_device()
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(uid, len(uid))
        rc = self.lib.h2o_rccl_init(ctypes.byref(h), self.world, buf, self.rank)
        if rc != 0:
            raise RuntimeError(f"ncclCommInitRank failed (rc={rc}, world={world}, rank={rank})")
        self.handle = h.value
        self.fn = ctypes.cast(self.lib.h2o_rccl_coll, ctypes.c_void_p).value
        self.ctx = self.handle

    def collective(self, op: int, send: torch.Tensor, recv: torch.Tensor, count: int, dtype: int) -> None:
        """One collective on the current stream (used by tests and by trainers outside the tree driver)."""
        rc = self.lib.h2o_rccl_coll(self.handle, op, send.data_ptr(), recv.data_ptr(), int(count), dtype,
                                    nat.stream_ptr())
        if rc != 0:
            raise RuntimeError(f"RCCL collective {op} failed (rc={rc})")

    def close(self):
        if self.handle:
            self.lib.h2o_rccl_destroy(self.handle, 0)
            self.handle = None


def _new_uid(lib) -> bytes:
    n = lib.h2o_rccl_id_bytes()
    buf = ctypes.create_string_buffer(n)
    rc = lib.h2o_rccl_unique_id(buf)
    if rc != 0:
        raise RuntimeError(f"ncclGetUniqueId failed (rc={rc})")
    return buf.raw


def native_comm(force: bool = False) -> NativeComm | None:
    """This process's RCCL communicator over the default process group (created on first use, collectively:
    every rank must call this at the same point), or None when the group does not run RCCL.

    ``force``: a communicator is wanted even without a multi-rank group — over a 1-rank ``nccl`` group, or a
    private 1-rank communicator when no group exists (the 1-GPU rehearsal of the sharded path)."""
    if os.environ.get("H2O_NATIVE_COMM") == "0" or not torch.cuda.is_available():
        return None
    have_pg = dist.is_available() and dist.is_initialized()
    if have_pg and dist.get_backend() != "nccl":
        return None
    if not have_pg and not force:
        return None
    world = dist.get_world_size() if have_pg else 1
    rank = dist.get_rank() if have_pg else 0
    from . import collectives as _coll
    if world == 1 and not (force or _coll.forced_sharded()):
        return None
    key = (world, rank, torch.cuda.current_device(), id(dist.group.WORLD) if have_pg else 0)
    with _lock:
        c = _comms.get(key)
        if c is not None:
            return c
        try:
            lib = load_rccl()
        except (OSError, RuntimeError) as e:   # no RCCL library (symmetric on every rank): torch's collectives
            import warnings
            warnings.warn(f"native RCCL communicator unavailable ({e}); tree exchange through torch.distributed")
            return None
        uid = _new_uid(lib) if rank == 0 else b""
        if world > 1:
            n = lib.h2o_rccl_id_bytes()
            t = torch.zeros(n, dtype=torch.uint8, device="cuda")
            if rank == 0:
                t.copy_(torch.frombuffer(bytearray(uid), dtype=torch.uint8))
            dist.broadcast(t, 0)
            uid = bytes(t.cpu().numpy().tobytes())
        c = NativeComm(world, rank, uid)
        _comms[key] = c
        return c


def reset():
    """Drop the cached communicators (tests that tear the process group down and build a new one)."""
    with _lock:
        for c in _comms.values():
            try:
                c.close()
            except Exception:  # noqa: BLE001
                pass
        _comms.clear()


_CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_void_p, ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p,
                       ctypes.c_longlong, ctypes.c_int, ctypes.c_void_p)


class HostTransport:
    """The native driver's collectives run by the process group's backend on host copies (gloo).

    The callback receives raw device pointers; they always point into the builder's own buffers, so each one
    is resolved to a byte view of a registered tensor."""

    def __init__(self, buffers: list):
        self.bufs = [(t.data_ptr(), t.numel() * t.element_size(), t) for t in buffers if t is not None]
        self._cb = _CB(self._call)          # keep the thunk alive for the builder's lifetime
        self.fn = ctypes.cast(self._cb, ctypes.c_void_p).value
        self.ctx = 0
        self.error = None

    def _view(self, ptr: int, nbytes: int, dtype) -> torch.Tensor:
        for base, size, t in self.bufs:
            if base <= ptr and ptr + nbytes <= base + size:
                off = ptr - base
                return t.view(-1).view(torch.uint8)[off:off + nbytes].view(dtype)
        raise RuntimeError(f"collective buffer {ptr:#x}+{nbytes} is not a registered builder buffer")

    def _call(self, ctx, op, send, recv, count, dtype, stream):
        try:
            dt = _DT[dtype]
            es = torch.tensor([], dtype=dt).element_size()
            W = coll.world()
            torch.cuda.current_stream().synchronize()
            if op == OP_ALLREDUCE:
                s = self._view(send, count * es, dt)
                r = self._view(recv, count * es, dt)
                if s.data_ptr() != r.data_ptr():
                    r.copy_(s)
                coll.all_reduce_(r)
            elif op == OP_REDUCE_SCATTER:
                coll.reduce_scatter_(self._view(recv, count * es, dt), self._view(send, W * count * es, dt))
            elif op == OP_ALLGATHER:
                coll.all_gather_into_(self._view(recv, W * count * es, dt), self._view(send, count * es, dt))
            else:
                return 1998
            torch.cuda.current_stream().synchronize()
            return 0
        except Exception as e:  # noqa: BLE001 - reported by the builder after the native call returns
            self.error = e
            return 1997
