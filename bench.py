#!/usr/bin/env python3
"""Bloom-filter build benchmark on MI355X (BASELINE.json metric: build keys/s + key-bytes GiB/s,
device-resident, 1/2/4/8 GPUs).

Default workload (N=1): BASELINE config 2 -- 100M x 16-byte keys, 10 bits/key
(m = 1,000,000,000 bits, k = 10), keys already resident in HBM.  One step = BloomFilter::new's
zeroed bit array (bf.rs:71) + build_filter_from_entries over the batch (bf.rs:126-128).
With N > 1 (torchrun, one rank per GPU) every rank builds its own independent SSTable shard
of the same size (config 4's compaction fan-in): weak scaling, no data-path collective.

Also: --config 3 (100M variable-length Zipf keys + 50M negative probes), --config 5 (1B x 32 B,
15 bits/key -> m saturates at u32::MAX, k = 4; keys split over ranks, OR all-reduce, full
probe sweep), --e2e (keys in host memory: H2D + build + D2H through the C ABI's pipeline).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import velarixdb_amd as vbf  # noqa: E402
from velarixdb_amd import workloads as wl  # noqa: E402
from velarixdb_amd._lib import call  # noqa: E402

HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: 8.0 TB/s spec
VALU_PEAK_LANE_OPS = 256 * 4 * 32 * 2.4e9  # 256 CUs x 4 SIMD32 x 2.4 GHz (int32 lane-ops/s)
# VALU lane-instructions per key of the build, from rocprofv3 SQ_INSTS_VALU (profiles/r01)
VALU_PER_KEY_CFG2 = 1611.0


def pmc_traffic(name):
    """Per-launch HBM bytes measured by tools/pmc_traffic.py from rocprofv3 PMC passes."""
    path = os.path.join(ROOT, "profiles", "r01", name)
    try:
        with open(path) as f:
            d = json.load(f)
        return d["per_launch_bytes"], "profiles/r01/" + name
    except (OSError, ValueError, KeyError):
        return None, None


def vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Ctx:
    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        # Rehearsal knobs for the N>1 path on a one-GPU box: VBF_SHARE_DEVICE=1 puts every rank
        # on cuda:0, VBF_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU).
        # The driver's multi-GPU runs set neither: one rank per GPU over RCCL.
        if os.environ.get("VBF_SHARE_DEVICE") == "1":
            self.local = 0
        self.backend = os.environ.get("VBF_DIST_BACKEND", "nccl")
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        if self.world > 1:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(self.backend)
        self.stream = torch.cuda.current_stream(self.dev)
        self.sp = ctypes.c_void_p(self.stream.cuda_stream)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def max_over_ranks(self, x):
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    def sum_over_ranks(self, x):
        if self.world == 1:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.SUM)
        return float(t.item())


def timed_steps(ctx, step, steps, warmup):
    """W untimed steps, then K steps bracketed by barrier + synchronize.

    Returns (max-over-ranks wall seconds, torch-event ms per step, library phase timings).
    The library brackets each kernel phase with hipEvents on the launch stream."""
    from velarixdb_amd._lib import lib, profile_read
    # Clock settle (untimed, on top of the W warmup steps): MI355X kernel durations keep
    # falling for the first ~25 ms of sustained load (k_tile_pack 4.6 -> 3.7 ms over its first
    # six launches under rocprofv3), so keep stepping until 0.3 s of work has run.
    t_settle = time.perf_counter()
    while True:
        step(None)
        torch.cuda.synchronize()
        if time.perf_counter() - t_settle > 0.3:
            break
    for _ in range(warmup):
        step(None)
    torch.cuda.synchronize()
    ctx.barrier()
    torch.cuda.synchronize()
    evs = []
    lib.vbf_profile_enable(1)
    profile_read()  # reset
    t0 = time.perf_counter()
    for _ in range(steps):
        step(evs)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    ctx.barrier()
    lib.vbf_profile_enable(0)
    phases = profile_read()
    kms = [a.elapsed_time(b) for a, b in evs]
    return ctx.max_over_ranks(t1 - t0), kms, phases


def time_probe_strategies(ctx, launch, reps=3):
    """Mean ms of one probe call per strategy (2 partitioned, 1 per-key gather), after a warm-up."""
    res = {}
    for strat, name in ((2, "partitioned"), (1, "gather")):
        launch(strat)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            launch(strat)
        torch.cuda.synchronize()
        res[name] = (time.perf_counter() - t0) / reps * 1e3
    return res


def phase_report(phases, steps):
    return {p: {"ms_per_launch": ms / n, "launches": n} for p, (ms, n) in phases.items() if n}


def cpu_baseline(keys_host, offsets_host, stride, n_sample, m, k, sample_desc, threads=1):
    """The oracle (a port of bf.rs:126-128 -> :84-92) on this node's host cores."""
    import oracle
    from velarixdb_amd.keys import HostBatch
    words = np.zeros((m + 31) // 32, np.uint32)
    b = HostBatch(keys_host, offsets_host, stride, n_sample, 1)
    t0 = time.perf_counter()
    oracle.build_words(b, m, k, words=words, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n_sample / dt, "unit": "keys/s", "cores": threads, "kind": "port",
            "sample": sample_desc, "seconds": round(dt, 3)}


# ---------------------------------------------------------------------------------------
def bench_fixed(ctx, args):
    """Configs 2 / 4: fixed 16-byte keys, 10 bits per key, one filter per rank."""
    n, L = args.keys, args.key_bytes
    p = wl.fpr_for_bits_per_key(args.bits_per_key)
    m, k = vbf.num_bits(n, p), vbf.num_hash_functions(vbf.num_bits(n, p), n)
    seed = wl.SEED_CFG2 if ctx.world == 1 else wl.SEED_CFG4 + ctx.rank
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", seed, 0, n, L, vp(keys), ctx.sp)
    nwords = (m + 31) // 32
    words = torch.empty(nwords, dtype=torch.int32, device=ctx.dev)

    def step(evs):
        words.zero_()  # BloomFilter::new: BitVec::from_elem(m, false) (bf.rs:71)
        if evs is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ctx.stream)
        call("vbf_build_dev_ex", vp(keys), None, L, n, 1, m, k, vp(words), args.strategy, ctx.sp)
        if evs is not None:
            b.record(ctx.stream)
            evs.append((a, b))

    wall, kms, phases = timed_steps(ctx, step, args.steps, args.warmup)

    # post-timing checks on the last build: every key present; fill ratio
    cnt = torch.zeros(1, dtype=torch.int64, device=ctx.dev)
    call("vbf_probe_count_dev", vp(keys), None, L, n, 1, m, k, vp(words), vp(cnt), ctx.sp)
    pop = torch.zeros(1, dtype=torch.int64, device=ctx.dev)
    call("vbf_popcount_dev", vp(words), nwords, vp(pop), ctx.sp)
    torch.cuda.synchronize()
    assert int(cnt.item()) == n, "false negatives: %d of %d keys found" % (cnt.item(), n)
    sweep = time_probe_strategies(ctx, lambda st: call("vbf_probe_count_dev_ex", vp(keys), None, L, n, 1, m, k,
                                                       vp(words), vp(cnt), st, ctx.sp))

    total_keys = ctx.sum_over_ranks(n) * args.steps
    value = total_keys / wall
    kavg = float(np.mean(kms)) / 1e3
    bytes_per_key = L + m / (8.0 * n)
    achieved = n * bytes_per_key / kavg / 1e9
    traffic, traffic_src = (pmc_traffic("traffic_config2.json") if (n, L, k) == (100_000_000, 16, 10)
                            and args.strategy != 1 else (None, None))
    res = {
        "metric": "Bloom build keys/s (device-resident keys, bit-exact SipHash-1-3 filter)",
        "value": value, "unit": "keys/s", "n_gpus": ctx.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "key_gib_per_s": value * L / 2**30,
        "config": {"workload": "config2: %dM x %dB keys per GPU, %d bits/key (m=%d, k=%d)%s" % (
            n // 10**6, L, args.bits_per_key, m, k,
            "" if ctx.world == 1 else
            "; %d independent SSTable shards, one per GPU (config 4's compaction fan-in, weak scaling)" % ctx.world),
            "n_keys_per_gpu": n, "key_bytes": L, "m_bits": m, "k": k, "len_prefix": True,
            "parallelism": "independent shards x%d" % ctx.world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_source": traffic_src,
                     "kernel": "build (all phases of one vbf_build_dev_ex launch)", "kernel_ms": kavg * 1e3,
                     "rocprof_kernels": {"tile_sort": "k_tile_pack<16, true, 10, true>", "transpose": "k_transpose_u16",
                                         "seg_or": "k_seg_or<3, 1024, 5>"},
                     "rocprof_summary": "profiles/r01/bench_default_kernel_stats.csv",
                     "valu_frac_est": n * VALU_PER_KEY_CFG2 / kavg / VALU_PEAK_LANE_OPS,
                     "algorithmic_bytes_per_key": bytes_per_key,
                     "siprounds_per_key": (L + 8) // 8 + 5 * k,
                     "phases": phase_report(phases, args.steps)},
        "fill_ratio": int(pop.item()) / m,
        "positive_sweep_ms": sweep,
    }
    if ctx.world == 1 and ctx.rank == 0 and not args.no_cpu_baseline:
        ns = args.cpu_sample
        host = keys[: ns * L].cpu().numpy()
        res["cpu_baseline"] = cpu_baseline(host, None, L, ns, m, k,
                                           "first %d of the %d keys, same m=%d/k=%d, 1 thread, ref-faithful "
                                           "(full SipHash per seed, u64 %%, serial like bf.rs:127)" % (ns, n, m, k))
        if args.cpu_opt_threads:
            t = args.cpu_opt_threads
            res["cpu_opt"] = cpu_baseline(host, None, L, ns, m, k, "same sample, prefix-shared, %d threads" % t, threads=t)
    return res


def bench_var(ctx, args):
    """Config 3: 100M variable-length (8..128 B Zipf) keys build + 50M negative probes."""
    n = args.keys
    p = wl.fpr_for_bits_per_key(args.bits_per_key)
    m = vbf.num_bits(n, p)
    k = vbf.num_hash_functions(m, n)
    off_h = wl.var_offsets(wl.SEED_CFG3, 0, n)
    off = torch.from_numpy(off_h.view(np.int64)).to(ctx.dev)
    keys = torch.empty(int(off_h[-1]), dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_var_dev", wl.SEED_CFG3, 0, n, vp(off), vp(keys), ctx.sp)
    nn = args.neg_keys
    noff_h = wl.var_offsets(wl.SEED_CFG3_NEG, 0, nn)
    noff = torch.from_numpy(noff_h.view(np.int64)).to(ctx.dev)
    nkeys = torch.empty(int(noff_h[-1]), dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_var_dev", wl.SEED_CFG3_NEG, 0, nn, vp(noff), vp(nkeys), ctx.sp)
    words = torch.empty((m + 31) // 32, dtype=torch.int32, device=ctx.dev)

    def step(evs):
        words.zero_()
        if evs is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ctx.stream)
        call("vbf_build_dev_ex", vp(keys), vp(off), 0, n, 1, m, k, vp(words), args.strategy, ctx.sp)
        if evs is not None:
            b.record(ctx.stream)
            evs.append((a, b))

    wall, kms, phases = timed_steps(ctx, step, args.steps, args.warmup)
    cnt = torch.zeros(1, dtype=torch.int64, device=ctx.dev)

    def probe(evs):
        cnt.zero_()
        if evs is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ctx.stream)
        call("vbf_probe_count_dev", vp(nkeys), vp(noff), 0, nn, 1, m, k, vp(words), vp(cnt), ctx.sp)
        if evs is not None:
            b.record(ctx.stream)
            evs.append((a, b))

    pwall, pkms, pphases = timed_steps(ctx, probe, args.steps, 1)
    fp = int(cnt.item())
    mean_len = float(off_h[-1]) / n
    value = ctx.sum_over_ranks(n) * args.steps / wall
    kavg = float(np.mean(kms)) / 1e3
    bpk = mean_len + 8 + m / (8.0 * n)
    achieved = n * bpk / kavg / 1e9
    return {
        "metric": "Bloom build keys/s (device-resident variable-length keys)", "value": value,
        "unit": "keys/s", "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "key_gib_per_s": value * mean_len / 2**30,
        "config": {"workload": "config3: %dM var-length keys (Zipf 8..128 B, mean %.1f B), %d bits/key (m=%d, k=%d) + %dM negative probes"
                   % (n // 10**6, mean_len, args.bits_per_key, m, k, nn // 10**6)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "partitioned build (offsets layout)",
                     "kernel_ms": kavg * 1e3, "algorithmic_bytes_per_key": bpk,
                     "phases": phase_report(phases, args.steps)},
        "probe": {"keys_per_s": nn / (float(np.mean(pkms)) / 1e3), "false_positives": fp,
                  "fpr": fp / nn, "kernel_ms": float(np.mean(pkms)),
                  "ms_by_strategy": time_probe_strategies(ctx, lambda st: call(
                      "vbf_probe_count_dev_ex", vp(nkeys), vp(noff), 0, nn, 1, m, k, vp(words), vp(cnt), st,
                      ctx.sp))},
    }


def bench_cfg5(ctx, args):
    """Config 5: 1B x 32 B keys, 15 bits/key (m saturates at u32::MAX, k = 4), split over ranks;
    partial filters OR-all-reduced; full positive probe sweep + negative FPR sample."""
    from velarixdb_amd.dist import or_allreduce_, padded_words, shard_range
    N, L = args.keys, 32
    p = wl.fpr_for_bits_per_key(15)
    m = vbf.num_bits(N, p)
    k = vbf.num_hash_functions(m, N)
    lo, hi = shard_range(N, ctx.rank, ctx.world)
    n = hi - lo
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", wl.SEED_CFG5, lo, n, L, vp(keys), ctx.sp)
    nwords = (m + 31) // 32
    buf, chunk = padded_words(nwords, ctx.world, ctx.dev)

    def step(evs):
        buf.zero_()
        if evs is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ctx.stream)
        call("vbf_build_dev_ex", vp(keys), None, L, n, 1, m, k, vp(buf), args.strategy, ctx.sp)
        if evs is not None:
            b.record(ctx.stream)
            evs.append((a, b))
        or_allreduce_(buf, chunk)

    wall, kms, phases = timed_steps(ctx, step, args.steps, args.warmup)
    cnt = torch.zeros(1, dtype=torch.int64, device=ctx.dev)
    t0 = time.perf_counter()
    call("vbf_probe_count_dev", vp(keys), None, L, n, 1, m, k, vp(buf), vp(cnt), ctx.sp)
    torch.cuda.synchronize()
    sweep = ctx.max_over_ranks(time.perf_counter() - t0)
    hits = int(ctx.sum_over_ranks(int(cnt.item())))
    assert hits == N, "positive sweep found %d of %d" % (hits, N)
    nn = args.neg_keys
    nk = torch.empty(nn * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", wl.SEED_CFG5 ^ 0xFF, N + ctx.rank * nn, nn, L, vp(nk), ctx.sp)
    cnt.zero_()
    call("vbf_probe_count_dev", vp(nk), None, L, nn, 1, m, k, vp(buf), vp(cnt), ctx.sp)
    torch.cuda.synchronize()
    fp = ctx.sum_over_ranks(int(cnt.item()))
    value = N * args.steps / wall
    return {
        "metric": "Bloom build keys/s (1B-key single filter across GPUs)", "value": value,
        "unit": "keys/s", "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic", "key_gib_per_s": value * L / 2**30,
        "config": {"workload": "config5: %d x 32B keys, 15 bits/key -> m=%d (u32-saturated), k=%d; OR all-reduce over %d ranks" % (N, m, k, ctx.world)},
        "build_kernel_ms": float(np.mean(kms)), "probe_sweep_keys_per_s": N / sweep,
        "negatives": {"n": nn * ctx.world, "false_positives": fp, "fpr": fp / (nn * ctx.world)},
    }


def bench_e2e(ctx, args):
    """Keys in host memory (memtable / compaction output): vbf_filter_set_host end to end."""
    n, L = args.keys, 16
    p = wl.fpr_for_bits_per_key(10)
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", wl.SEED_CFG2, 0, n, L, vp(keys), ctx.sp)
    host = keys.cpu().numpy()
    del keys
    from velarixdb_amd.keys import HostBatch
    hb = HostBatch(host, None, L, n, 1)
    times = []
    for i in range(args.warmup + args.steps):
        t0 = time.perf_counter()
        bf = vbf.BloomFilter(p, n, device=ctx.local)
        bf.set_batch(hb)
        w = bf.words()  # D2H of the finished filter (written back with the SST)
        t1 = time.perf_counter()
        if i >= args.warmup:
            times.append(t1 - t0)
        del bf
    t = float(np.median(times))
    return {"metric": "Bloom build keys/s end-to-end (host keys: H2D + build + D2H)", "value": n / t,
            "unit": "keys/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": t * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64", "data": "synthetic", "config": {"workload": "config2 e2e %dM x 16B, filter %d words" % (n // 10**6, w.size)}}


def bench_sst(ctx, args):
    """the lazy filter rebuild of range.rs:117-128 from a config-2 SST --
    data.db decode (fs/mod.rs:275-332) alone, and decode + build fused
    (vbf_filter_rebuild_from_sst_dev).  data.db is device-resident (as a GPU-direct read would
    leave it); each step includes the decoder's one entry-count readback."""
    n, L = args.keys, 16
    per = 4096 // (L + 17)
    nb = (n + per - 1) // per
    data = torch.empty(n * (L + 17), dtype=torch.uint8, device=ctx.dev)
    blocks = torch.empty(nb, dtype=torch.int32, device=ctx.dev)
    call("vbf_gen_sst_fixed_dev", wl.SEED_CFG2, 0, n, L, vp(data), vp(blocks), ctx.sp)
    out_k = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    out_o = torch.empty(n + 1, dtype=torch.int64, device=ctx.dev)
    got = ctypes.c_uint64()

    def decode(evs):
        call("vbf_sst_decode_dev", vp(data), data.numel(), vp(blocks), nb, vp(out_k), out_k.numel(), vp(out_o),
             None, None, None, n + 1, ctypes.byref(got), ctx.sp)

    dwall, _, dph = timed_steps(ctx, decode, args.steps, args.warmup)
    assert got.value == n
    p = wl.fpr_for_bits_per_key(10)
    bf = vbf.BloomFilter(p, n, device=ctx.local)

    def rebuild(evs):
        bf.rebuild_from_sst_dev(vp(data), data.numel(), vp(blocks), nb, ctx.sp)

    rwall, _, rph = timed_steps(ctx, rebuild, args.steps, args.warmup)
    res = {"metric": "SST filter rebuild keys/s (data.db decode + build, device-resident data.db)",
           "value": ctx.sum_over_ranks(n) * args.steps / rwall, "unit": "keys/s", "n_gpus": ctx.world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": rwall / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64",
           "data": "synthetic",
           "config": {"workload": "config2 SST: %dM x 16B keys in data.db (%.2f GB, %d blocks), m=%d, k=%d"
                      % (n // 10**6, data.numel() / 1e9, nb, bf.num_bits(), bf.no_of_hash_func)},
           "decode_only": {"ms_per_step": dwall / args.steps * 1e3,
                           "entries_per_s": n * args.steps / dwall,
                           "data_gb_per_s": data.numel() * args.steps / dwall / 1e9,
                           "phases": phase_report(dph, args.steps)},
           "phases": phase_report(rph, args.steps)}
    if ctx.world == 1 and ctx.rank == 0 and not args.no_cpu_baseline:
        import oracle
        ns = min(n, args.cpu_sample)
        host = data[: ns * (L + 17)].cpu().numpy()
        t0 = time.perf_counter()
        keys, offs, *_ = oracle.sst_decode(host)
        from velarixdb_amd.keys import HostBatch
        oracle.build_words(HostBatch(keys, offs, 0, ns, 1), bf.num_bits(), bf.no_of_hash_func)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": ns / dt, "unit": "keys/s", "cores": 1, "kind": "port",
                               "sample": "first %d entries of the same data.db: load_entries + build" % ns,
                               "seconds": round(dt, 3)}
    return res


def bench_compact(ctx, args):
    """one bucket of 4 sorted tables x 25M 16-byte keys (half of each table's
    keys also in another table, 5 % tombstones) through the fold (vbf_compact_merge_dev), then the
    gather into the build's layout and the merged table's filter build (sized.rs:170-200)."""
    nr, per = 4, args.keys // 4
    L = 16
    j = torch.arange(per, device=ctx.dev, dtype=torch.int64)
    ks, cr, tb = [], [], []
    g = torch.Generator(device=ctx.dev)
    g.manual_seed(7)
    for r in range(nr):
        v = 2 * j + (r % 2) + (per * (r // 2))  # tables 0/2 and 1/3 overlap by half
        be = v.view(torch.uint8).view(-1, 8).flip(1)
        ks.append(torch.cat([be, be], dim=1).reshape(-1))
        cr.append(torch.randint(0, 1 << 40, (per,), device=ctx.dev, generator=g))
        tb.append((torch.rand(per, device=ctx.dev, generator=g) < 0.05).to(torch.uint8))
    keys, created, tomb = torch.cat(ks), torch.cat(cr), torch.cat(tb)
    offs = torch.arange(nr * per + 1, device=ctx.dev, dtype=torch.int64) * L
    run_off = (np.arange(nr + 1, dtype=np.uint64) * per)
    ids = torch.empty(nr * per, dtype=torch.int32, device=ctx.dev)
    mk = torch.empty(nr * per * L, dtype=torch.uint8, device=ctx.dev)
    mo = torch.empty(nr * per + 1, dtype=torch.int64, device=ctx.dev)
    n, nu, kb = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()

    def merge(evs):
        call("vbf_compact_merge_dev", vp(keys), vp(offs), vp(created), vp(tomb), run_off.ctypes.data, nr,
             None, None, None, 0, 0, 0, 10**15, 1 << 41, vp(ids), ctypes.byref(n), None, None,
             ctypes.byref(nu), ctx.sp)

    mwall, _, mph = timed_steps(ctx, merge, args.steps, args.warmup)
    bf = vbf.BloomFilter(1e-4, max(n.value, 1), device=ctx.local)

    def full(evs):
        merge(evs)
        call("vbf_gather_entries_dev", vp(keys), vp(offs), None, None, None, vp(ids), n.value, vp(mk), mk.numel(),
             vp(mo), None, None, None, ctypes.byref(kb), ctx.sp)
        bf.set_dev(vp(mk), None, L, n.value, 1, ctx.sp)

    fwall, _, fph = timed_steps(ctx, full, args.steps, args.warmup)
    total = nr * per
    res = {"metric": "compaction merge entries/s (4 sorted tables -> merged table + its filter, device-resident)",
           "value": ctx.sum_over_ranks(total) * args.steps / fwall, "unit": "entries/s", "n_gpus": ctx.world,
           "steps": args.steps, "warmup": args.warmup, "ms_per_step": fwall / args.steps * 1e3,
           "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
           "config": {"workload": "bucket of %d tables x %dM x 16B keys, %d merged entries" % (nr, per // 10**6, n.value)},
           "merge_only": {"ms_per_step": mwall / args.steps * 1e3, "entries_per_s": total * args.steps / mwall,
                          "phases": phase_report(mph, args.steps)},
           "phases": phase_report(fph, args.steps)}
    if ctx.world == 1 and ctx.rank == 0 and not args.no_cpu_baseline:
        import oracle
        ns = min(per, args.cpu_sample // nr)
        hk = np.concatenate([k.view(-1, L)[:ns].cpu().numpy().reshape(-1) for k in ks])
        ho = np.arange(nr * ns + 1, dtype=np.uint64) * L
        hc = np.concatenate([c[:ns].cpu().numpy() for c in cr])
        ht = np.concatenate([t[:ns].cpu().numpy() for t in tb])
        t0 = time.perf_counter()
        oracle.compact_merge(hk, ho, hc, ht, np.arange(nr + 1, dtype=np.uint64) * ns, False, 0, 10**15, 1 << 41)
        dt = time.perf_counter() - t0
        res["cpu_baseline"] = {"value": nr * ns / dt, "unit": "entries/s", "cores": 1, "kind": "port",
                               "sample": "first %d entries of each table: the pairwise fold only" % ns,
                               "seconds": round(dt, 3)}
    return res


def bench_multi(ctx, args):
    """100M device-resident 16-byte keys probed against 8 SST filters (each
    10M keys at 10 bits/key) in one launch -- key-range test + contains() per (key, SST)."""
    n, L, S = args.keys, 16, 8
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", wl.SEED_CFG2, 0, n, L, vp(keys), ctx.sp)
    p = wl.fpr_for_bits_per_key(10)
    filters = []
    for s_ in range(S):
        f = vbf.BloomFilter(p, 10_000_000, device=ctx.local)
        f.set_dev(vp(keys[s_ * 10_000_000 * L:]), None, L, 10_000_000, 1, ctx.sp)
        filters.append(f)
    handles = (ctypes.c_void_p * S)(*[f._h.value for f in filters])
    out = torch.empty(n * S, dtype=torch.uint8, device=ctx.dev)

    def step(evs):
        call("vbf_multi_probe_dev", vp(keys), None, L, n, 1, S, handles, None, None, vp(out), ctx.sp)

    wall, _, _ = timed_steps(ctx, step, args.steps, args.warmup)
    hits = int(out.view(n, S).any(dim=1).sum().item())
    return {"metric": "multi-SST probe keys/s (each key tested against 8 filters, device-resident)",
            "value": ctx.sum_over_ranks(n) * args.steps / wall, "unit": "keys/s", "n_gpus": ctx.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "%dM x 16B keys vs %d filters of 10M keys (m=1e8, k=10); %d keys hit some SST"
                       % (n // 10**6, S, hits)},
            "probes_per_s": ctx.sum_over_ranks(n) * S * args.steps / wall}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=2, choices=[2, 3, 4, 5])
    ap.add_argument("--keys", type=int, default=None)
    ap.add_argument("--key-bytes", type=int, default=16)
    ap.add_argument("--bits-per-key", type=int, default=10)
    ap.add_argument("--neg-keys", type=int, default=None)
    ap.add_argument("--e2e", action="store_true")
    ap.add_argument("--sst", action="store_true", help="SST data.db decode + rebuild (8(f) row 2)")
    ap.add_argument("--compact", action="store_true", help="compaction merge + filter (8(f) row 3)")
    ap.add_argument("--multi", action="store_true", help="batched multi-SST probe (8(f) row 4)")
    ap.add_argument("--strategy", type=int, default=0, help="0 auto, 1 atomic, 2 partitioned")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=10_000_000)
    ap.add_argument("--cpu-opt-threads", type=int, default=16)
    args = ap.parse_args()
    ctx = Ctx(args)
    if args.config == 5:
        args.keys = args.keys or 1_000_000_000
        args.neg_keys = args.neg_keys or 10_000_000
        res = bench_cfg5(ctx, args)
    elif args.config == 3:
        args.keys = args.keys or 100_000_000
        args.neg_keys = args.neg_keys or 50_000_000
        res = bench_var(ctx, args)
    elif args.compact:
        args.keys = args.keys or 100_000_000
        res = bench_compact(ctx, args)
    elif args.multi:
        args.keys = args.keys or 100_000_000
        res = bench_multi(ctx, args)
    elif args.sst:
        args.keys = args.keys or 100_000_000
        res = bench_sst(ctx, args)
    elif args.e2e:
        args.keys = args.keys or 100_000_000
        res = bench_e2e(ctx, args)
    else:
        args.keys = args.keys or (100_000_000 if args.config == 2 else 50_000_000)
        res = bench_fixed(ctx, args)
    if ctx.rank == 0:
        print(json.dumps(res), flush=True)
    if ctx.world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
