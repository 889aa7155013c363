"""Device-resident batch API (the hot path): many chunks, one launch sequence.

Replaces N calls of ``DefaultChunk::read_chunk_into`` (chunk.rs:288-301) /
``write_chunk`` (chunk.rs:306-323) with ``zcg_decode_batch`` /
``zcg_encode_batch`` over device buffers.  torch provides device memory and
the stream (plumbing only); the kernels are the HIP ones in ``csrc/``.
"""
from __future__ import annotations

import ctypes
from typing import List, Sequence, Tuple

import numpy as np

from . import _native
from .chunk import _raise_status, abi_array
from .metadata import ArrayMetadata

ALIGN = 256


def _torch():
    import torch
    return torch


class PackedStreams:
    """Compressed chunk streams packed into ONE device buffer (256-B aligned
    slots) plus the device ``zcg_chunk`` descriptor array."""

    def __init__(self, streams: Sequence[bytes], dst_bytes: int, device, dst=None,
                 slot_copies: int = 1):
        torch = _torch()
        n_unique = len(streams)
        offs, pos = [], 0
        for s in streams:
            offs.append(pos)
            pos += (len(s) + ALIGN - 1) // ALIGN * ALIGN
        host = np.zeros(max(pos, ALIGN), np.uint8)
        for o, s in zip(offs, streams):
            host[o:o + len(s)] = np.frombuffer(s, np.uint8)
        self.src = torch.from_numpy(host).to(device)
        self.n = n_unique * slot_copies
        self.dst_bytes = dst_bytes
        self.dst = dst if dst is not None else torch.empty(max(self.n * dst_bytes, 1), dtype=torch.uint8,
                                                           device=device)
        base = self.src.data_ptr()
        dbase = self.dst.data_ptr()
        desc = np.zeros((self.n, 4), np.uint64)
        for i in range(self.n):
            u = i % n_unique
            desc[i] = (base + offs[u], len(streams[u]), dbase + i * dst_bytes, dst_bytes)
        self.src_lens = np.array([len(streams[i % n_unique]) for i in range(self.n)], np.uint64)
        self.desc = torch.from_numpy(desc.view(np.int64)).to(device)
        self.status = torch.full((self.n,), -1, dtype=torch.int32, device=device)

    def compressed_bytes(self) -> int:
        return int(self.src_lens.sum())


class BatchCodec:
    def __init__(self, device: int = 0):
        self.ctx = _native.context(device)
        self.device = device

    def decode(self, meta: ArrayMetadata, packed: PackedStreams, stream=None, flags: int = 0):
        """Enqueue the batch decode on `stream` (torch stream or raw handle)."""
        torch = _torch()
        arr = abi_array(meta, flags)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        h = s.cuda_stream if hasattr(s, "cuda_stream") else int(s)
        r = self.ctx.lib.zcg_decode_batch(self.ctx.handle, ctypes.byref(arr), packed.desc.data_ptr(),
                                          packed.n, packed.status.data_ptr(), h)
        _raise_status(r, self.ctx, "decode_batch")

    def encode(self, meta: ArrayMetadata, desc, n: int, out_len, status, stream=None):
        torch = _torch()
        arr = abi_array(meta)
        s = stream if stream is not None else torch.cuda.current_stream(self.device)
        h = s.cuda_stream if hasattr(s, "cuda_stream") else int(s)
        r = self.ctx.lib.zcg_encode_batch(self.ctx.handle, ctypes.byref(arr), desc.data_ptr(), n,
                                          out_len.data_ptr(), status.data_ptr(), h)
        _raise_status(r, self.ctx, "encode_batch")

    def encode_bound(self, meta: ArrayMetadata, nbytes: int) -> int:
        arr = abi_array(meta)
        return int(self.ctx.lib.zcg_encode_bound(ctypes.byref(arr.compression), nbytes))


def make_encode_batch(elems, n: int, dst_cap: int, device):
    """Descriptors for encoding n chunks stored back to back in `elems`
    (device uint8 tensor of n*D bytes) into n slots of dst_cap bytes."""
    torch = _torch()
    D = elems.numel() // n
    dst = torch.empty(n * dst_cap, dtype=torch.uint8, device=device)
    desc = np.zeros((n, 4), np.uint64)
    for i in range(n):
        desc[i] = (elems.data_ptr() + i * D, D, dst.data_ptr() + i * dst_cap, dst_cap)
    d = torch.from_numpy(desc.view(np.int64)).to(device)
    out_len = torch.zeros(n, dtype=torch.int64, device=device)
    status = torch.full((n,), -1, dtype=torch.int32, device=device)
    return d, dst, out_len, status
