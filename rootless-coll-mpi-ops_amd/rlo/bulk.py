"""Bulk (large-message) rootless bcast over a world's parts (rlo_bulk_* in rlo_hip.h).

    b = Bulk(world, buf_bytes)          # this part's ranks' receive buffers (HBM, uncached)
    blobs = exchange(b.export())        # every part's blob, in part order
    b.connect(blobs)
    b.tensor(rank)[:n].copy_(payload)   # the originator's message, in its own buffer
    b.reset(); <host barrier>; b.launch(origin, n); b.wait()   # on every part
"""
import ctypes

from . import _lib as L
from ._lib import check


def plan(n, nbytes, chunk=0, blocks=0, cross_gpu=False):
    """rlo_bulk_plan: the geometry rlo_bulk_launch would use (host arithmetic, no GPU needed)"""
    lib = L.load()
    out = L.BulkPlan()
    check(lib.rlo_bulk_plan(n, nbytes, chunk, blocks, 1 if cross_gpu else 0, ctypes.byref(out)), "rlo_bulk_plan")
    return {"stripe": out.stripe, "chunk": out.chunk, "nchunks": out.nchunks, "blocks": out.blocks}


class _CAI:
    def __init__(self, ptr, nbytes):
        self.__cuda_array_interface__ = {"shape": (nbytes,), "typestr": "|u1", "data": (ptr, False), "version": 3}


class Bulk:
    def __init__(self, world, buf_bytes):
        self.lib = L.load()
        self.world = world
        self.buf_bytes = buf_bytes
        h = ctypes.c_void_p()
        check(self.lib.rlo_bulk_create(world.h, buf_bytes, ctypes.byref(h)), "rlo_bulk_create")
        self.h = h

    def export(self):
        buf = ctypes.create_string_buffer(L.RLO_BULK_BLOB_BYTES)
        check(self.lib.rlo_bulk_export(self.h, buf, L.RLO_BULK_BLOB_BYTES), "rlo_bulk_export")
        return buf.raw

    def connect(self, blobs):
        check(self.lib.rlo_bulk_connect(self.h, b"".join(blobs), len(blobs)), "rlo_bulk_connect")

    def tensor(self, rank):
        """a uint8 torch view of a local rank's receive buffer (zero copy)"""
        import torch

        ptr = self.lib.rlo_bulk_buffer(self.h, rank)
        if not ptr:
            raise L.RloError("rank %d is not local" % rank)
        return torch.as_tensor(_CAI(ptr, self.buf_bytes), device="cuda")

    def reset(self, stream=None):
        check(self.lib.rlo_bulk_reset(self.h, stream), "rlo_bulk_reset")

    def launch(self, origin, nbytes, blocks=0, chunk=0, stream=None):
        """blocks 0 / chunk 0: sized by the library (rlo_bulk_launch in rlo_hip.h)"""
        check(self.lib.rlo_bulk_launch(self.h, origin, nbytes, chunk, blocks, stream), "rlo_bulk_launch")

    def wait(self, raise_on_error=True):
        """kernel ms; with raise_on_error=False, (ms, rc) so that SPMD callers stay in step"""
        ms = ctypes.c_float()
        rc = self.lib.rlo_bulk_wait(self.h, ctypes.byref(ms))
        if not raise_on_error:
            return ms.value, rc
        check(rc, "rlo_bulk_wait")
        return ms.value

    def close(self):
        if self.h:
            self.lib.rlo_bulk_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()
