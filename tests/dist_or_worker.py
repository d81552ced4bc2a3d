"""One rank of the config-5 exchange rehearsal (tests/test_gpu_dist.py): launched by
torch.distributed.run with every rank on cuda:0 and a gloo group (RCCL refuses two ranks on one
GPU).  Rank r builds its contiguous shard of the keys into a full-width partial filter (fresh
partitioned build), the partials are merged by velarixdb_amd.dist.or_allreduce_ (host-staged
gloo exchange, HIP OR fold), and every rank writes its merged words to OUT.rank<r>.npy.

usage: python -m torch.distributed.run ... dist_or_worker.py N L M K SEED OUT"""
import ctypes
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    n, L, m, k, seed = (int(x, 0) for x in sys.argv[1:6])
    out = sys.argv[6]
    dist.init_process_group("gloo")
    rank, world = dist.get_rank(), dist.get_world_size()
    import velarixdb_amd  # noqa: F401
    from velarixdb_amd._lib import call
    from velarixdb_amd.dist import or_allreduce_, padded_words, shard_range
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    sp = ctypes.c_void_p(torch.cuda.current_stream(dev).cuda_stream)
    lo, hi = shard_range(n, rank, world)
    keys = torch.empty((hi - lo) * L, dtype=torch.uint8, device=dev)
    call("vbf_gen_fixed_dev", seed, lo, hi - lo, L, ctypes.c_void_p(keys.data_ptr()), sp)
    nwords = (m + 31) // 32
    buf, chunk = padded_words(nwords, world, dev)
    buf.fill_(-1)  # garbage: the fresh build writes every word of its filter
    call("vbf_build_dev_ex", ctypes.c_void_p(keys.data_ptr()), None, L, hi - lo, 1, m, k,
         ctypes.c_void_p(buf.data_ptr()), 2 | 0x100, sp)
    buf[nwords:] = 0
    torch.cuda.synchronize()
    or_allreduce_(buf, chunk)
    torch.cuda.synchronize()
    np.save(out + ".rank%d.npy" % rank, buf[:nwords].cpu().numpy().view(np.uint32))
    dist.barrier()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
