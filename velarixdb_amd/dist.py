"""Multi-GPU layout of the Bloom-filter path.  One process per GPU.

* Independent SSTables (compaction fan-in, compactors/sized.rs:170-200): each rank builds its
  own shard's filter.  No data-path collective -- weak scaling.
* One filter over a key set split across ranks (BASELINE config 5): each rank ORs its keys
  into a full-width partial array, then the partials are merged with a bitwise-OR
  all-reduce.  RCCL has no OR reduction, so it is composed from data movement plus a local
  OR: all_to_all_single (rank r receives every rank's copy of bit-range r: a reduce-scatter
  by bit range), the OR of those copies in one pass (HIP kernel vbf_or_fold_dev: each copy read
  once, the result written once, into the receive buffer's first slice), then
  all_gather_into_tensor so every rank holds the full filter for its probe sweep.  The receive
  buffer is one workspace per (device, size), reused across calls.
"""
import ctypes

import torch
import torch.distributed as dist

from ._lib import call


def shard_range(n, rank, world):
    """Contiguous [lo, hi) of n items for `rank`: sizes differ by at most one."""
    lo = n * rank // world
    hi = n * (rank + 1) // world
    return lo, hi


def or_words_dev(acc, src):
    """acc |= src on the GPU (HIP kernel vbf_or_words_dev); same-shape int32 device tensors."""
    if acc.device.type != "cuda" or src.device.type != "cuda":
        raise ValueError("or_words_dev needs device tensors (the OR runs as a HIP kernel)")
    if acc.device != src.device:
        raise ValueError("or_words_dev: acc on %s, src on %s" % (acc.device, src.device))
    if acc.dtype != torch.int32 or src.dtype != torch.int32:
        raise ValueError("or_words_dev needs int32 words (got %s, %s)" % (acc.dtype, src.dtype))
    if acc.shape != src.shape:
        raise ValueError("or_words_dev: shapes differ (%s vs %s)" % (tuple(acc.shape), tuple(src.shape)))
    if not (acc.is_contiguous() and src.is_contiguous()):
        raise ValueError("or_words_dev needs contiguous tensors")
    stream = ctypes.c_void_p(torch.cuda.current_stream(acc.device).cuda_stream)
    call("vbf_or_words_dev", ctypes.c_void_p(acc.data_ptr()), ctypes.c_void_p(src.data_ptr()), acc.numel(), stream)


def padded_words(nwords, world, device):
    """An int32 buffer for nwords words padded so each rank's bit range is 16-B aligned."""
    chunk = -(-nwords // world)
    chunk = (chunk + 3) // 4 * 4
    return torch.zeros(chunk * world, dtype=torch.int32, device=device), chunk


def or_fold_dev(dst, parts, nparts, chunk):
    """dst = parts[0:chunk] | parts[chunk:2 chunk] | ... (nparts slices) in one HIP pass
    (vbf_or_fold_dev); dst may be parts[:chunk] itself.  int32 device tensors."""
    for t in (dst, parts):
        if t.device.type != "cuda" or t.dtype != torch.int32 or not t.is_contiguous():
            raise ValueError("or_fold_dev needs contiguous int32 device tensors")
    if dst.device != parts.device:
        raise ValueError("or_fold_dev: dst on %s, parts on %s" % (dst.device, parts.device))
    if dst.numel() != chunk or parts.numel() < nparts * chunk:
        raise ValueError("or_fold_dev: dst holds %d words, parts %d (want %d and %d x %d)"
                         % (dst.numel(), parts.numel(), chunk, nparts, chunk))
    stream = ctypes.c_void_p(torch.cuda.current_stream(dst.device).cuda_stream)
    call("vbf_or_fold_dev", ctypes.c_void_p(dst.data_ptr()), ctypes.c_void_p(parts.data_ptr()), chunk, nparts,
         chunk, stream)


def or_fold_host(dst, parts, nparts, chunk):
    """The same fold on CPU tensors (the gloo tests of the exchange)."""
    acc = parts[:chunk].clone()
    for r in range(1, nparts):
        acc.bitwise_or_(parts[r * chunk:(r + 1) * chunk])
    dst.copy_(acc)


_recv = {}


def _recv_buffer(like):
    """The all_to_all receive buffer: one per (device, dtype, size), kept for the next call (config 5:
    a 512 MiB array per rank per step)."""
    key = (str(like.device), like.dtype, like.numel())
    t = _recv.get(key)
    if t is None:
        t = torch.empty_like(like)
        _recv[key] = t
    return t


def or_allreduce_(buf, chunk, group=None, fold=None):
    """In place: buf (padded_words layout) becomes the OR of every rank's buf.  The fold is the HIP
    kernel for device tensors (or_fold_dev), or `fold` (the CPU gloo tests pass or_fold_host).

    Device words under a gloo group (the one-GPU rehearsal of the N > 1 path, where RCCL refuses
    two ranks on one card) move through host tensors for gloo's all_to_all / all_gather, while
    the fold stays on the GPU: the same HIP kernel the RCCL path runs."""
    if not dist.is_initialized():
        return buf
    world = dist.get_world_size(group)
    if world == 1:
        return buf
    if fold is None:
        fold = or_fold_dev if buf.device.type == "cuda" else or_fold_host
    staged = buf.device.type == "cuda" and dist.get_backend(group) == "gloo"
    src = buf.cpu() if staged else buf
    recv = _recv_buffer(src)
    dist.all_to_all_single(recv, src, group=group)
    parts = recv.to(buf.device) if staged else recv
    acc = parts[:chunk]
    fold(acc, parts, world, chunk)  # into the first slice: every copy read once
    if staged:
        full = torch.empty_like(src)
        dist.all_gather_into_tensor(full, acc.cpu(), group=group)
        buf.copy_(full)
    else:
        dist.all_gather_into_tensor(buf, acc, group=group)
    return buf
