#!/usr/bin/env python3
"""Bloom-filter build benchmark on MI355X (BASELINE.json metric: build keys/s + key-bytes GiB/s,
device-resident, 1/2/4/8 GPUs).

Default workload at N=1: BASELINE config 2 -- 100M x 16-byte keys, 10 bits/key
(m = 1,000,000,000 bits, k = 10), keys already resident in HBM.  One step = BloomFilter::new's
zeroed bit array (bf.rs:71) + build_filter_from_entries over the batch (bf.rs:126-128).
At N > 1 the default is BASELINE config 4, the compaction fan-in: every rank builds its own
independent SSTable shard of 50M x 16-byte keys (m = 500,000,000, k = 10, seed 0x5EED0040 +
rank), one filter per merged table as compactors/sized.rs:170-200 builds them (filter at
:192-193).  Weak scaling, no data-path collective.

`python bench.py --gpus N` with N > 1 and no launcher in the environment starts the N ranks
itself (torch.distributed.run as a child process, before anything touches the GPU) and exits
with their status.  Under a launcher, WORLD_SIZE must equal --gpus.

Also: --config 3 (100M variable-length Zipf keys + 50M negative probes), --config 5 (1B x 32 B,
15 bits/key -> m saturates at u32::MAX, k = 4; keys split over ranks, OR all-reduce, full
probe sweep), --e2e (keys in host memory: H2D + build + D2H through the C ABI's pipeline).
"""
import argparse
import ctypes
import json
import os
import socket
import subprocess
import sys
import time


def make_parser():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None,
                    help="ranks, one per GPU (default: WORLD_SIZE under a launcher, else 1)")
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--config", type=int, default=None, choices=[2, 3, 4, 5],
                    help="BASELINE config (default: 2 on one GPU, 4 on several)")
    ap.add_argument("--keys", type=int, default=None)
    ap.add_argument("--key-bytes", type=int, default=16)
    ap.add_argument("--bits-per-key", type=int, default=10)
    ap.add_argument("--raw-keys", action="store_true",
                    help="configs 2/4: hash the keys without the length prefix (len_prefix = 0: pre-encoded "
                         "integer keys such as bf.rs:307-424's usize keys)")
    ap.add_argument("--neg-keys", type=int, default=None)
    ap.add_argument("--probe-ab", action="store_true",
                    help="config 5: also time the positive sweep on the round-3 probe pipeline (VBF_PROBE_PU=0)")
    ap.add_argument("--e2e", action="store_true")
    ap.add_argument("--e2e-fresh-out", action="store_true", help="--e2e: a fresh host array per step")
    ap.add_argument("--sst", action="store_true", help="SST data.db decode + rebuild (8(f) row 2)")
    ap.add_argument("--compact", action="store_true", help="compaction merge + filter (8(f) row 3)")
    ap.add_argument("--multi", action="store_true", help="batched multi-SST probe (8(f) row 4)")
    ap.add_argument("--fanout", action="store_true",
                    help="the compaction loop (sized.rs:170-200): per-bucket builds, synchronous vs asynchronous")
    ap.add_argument("--buckets", type=int, default=8)
    ap.add_argument("--fanout-reuse", action="store_true", help="--fanout: no per-bucket materialisation")
    ap.add_argument("--memtable", action="store_true",
                    help="single-key set/contains latency on a memtable-size filter (mem.rs:207-230)")
    ap.add_argument("--strategy", type=int, default=0, help="0 auto, 1 atomic, 2 partitioned")
    ap.add_argument("--separate-zero", action="store_true",
                    help="zero the filter with a fill kernel before each build instead of VBF_BUILD_FRESH")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", type=int, default=10_000_000)
    ap.add_argument("--cpu-opt-threads", type=int, default=None,
                    help="threads of the prefix-shared CPU port (default: every usable host core)")
    ap.add_argument("--plan-only", action="store_true",
                    help="launch the ranks, report world size and each rank's workload, touch no GPU")
    return ap


def launch_plan(gpus, env):
    """How this invocation runs: ("spawn", N) -- no launcher and --gpus N > 1, so start N ranks;
    ("run", world) -- run this process as one rank of `world`.  A launcher's WORLD_SIZE that
    disagrees with an explicit --gpus is an error (the driver's N must be the N measured)."""
    ws = env.get("WORLD_SIZE")
    if ws is None:
        n = 1 if gpus is None else gpus
        if n < 1:
            raise ValueError("--gpus must be >= 1 (got %d)" % n)
        return ("spawn", n) if n > 1 else ("run", 1)
    world = int(ws)
    if gpus is not None and gpus != world:
        raise ValueError("--gpus %d but the launcher started WORLD_SIZE=%d ranks" % (gpus, world))
    return ("run", world)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def spawn_command(nproc, argv, port):
    """torch.distributed.run over this script, one rank per GPU, rendezvous on 127.0.0.1."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(nproc),
            "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)


def maybe_spawn_ranks():
    """Runs before torch or libvbf touch the GPU: a child process, never an exec."""
    args, _ = make_parser().parse_known_args()
    mode, n = launch_plan(args.gpus, os.environ)
    if mode == "spawn":
        print("bench.py: starting %d ranks (torch.distributed.run, one per GPU)" % n, file=sys.stderr, flush=True)
        rc = subprocess.call(spawn_command(n, sys.argv[1:], _free_port()))
        sys.exit(rc)


if __name__ == "__main__":
    maybe_spawn_ranks()

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


# rocprofv3 names of the build's kernels, and the summary of the same command, per (key bytes, k)
ROCPROF = {
    (16, 10): ({"tile_sort": "k_tile_pack<16, true, 10, true, false, 1, 0, 20, 0, false>",
                "seg_or": "k_seg_or<7, 1024, 5, 8>"}, "profiles/r06/bench_default_kernel_stats.csv"),
    (16, 19): ({"tile_sort": "k_tile_pack<16, true, 19, true, false, 1, 0, 20, 0, false>",
                "seg_or": "k_seg_or<7, 1024, 4, 8>"}, "profiles/r06/bench_k19_kernel_stats.csv"),
}


SQ_FILES = {10: "sq_tile_pack.json", 19: "sq_tile_pack_k19.json"}


def pmc_sq(name, keys):
    """VALU issue busy, wait fractions and VALU lane-instructions per key of k_tile_pack from one
    rocprofv3 SQ pass (tools/pmc_sq.py) over a build of `keys` keys; the newest round's."""
    for rnd in ("r06", "r05", "r04", "r03", "r02"):
        path = os.path.join(ROOT, "profiles", rnd, name)
        try:
            with open(path) as f:
                d = json.load(f)
            return {"valu_issue_busy": d["valu_issue_busy"], "wave_wait_any_frac": d["wave_wait_any_frac"],
                    "valu_lane_instr_per_key": d["counters_per_dispatch"]["SQ_INSTS_VALU"] * 64 / keys,
                    "source": "profiles/%s/%s" % (rnd, name)}
        except (OSError, ValueError, KeyError):
            continue
    return None


def pmc_traffic(name, kernel=None):
    """HBM bytes measured by tools/pmc_traffic.py from rocprofv3 PMC passes (the newest round's
    measurement): (one launch of `kernel` -- read + write --, one whole build, source file)."""
    for rnd in ("r06", "r05", "r04", "r03", "r02", "r01"):
        path = os.path.join(ROOT, "profiles", rnd, name)
        try:
            with open(path) as f:
                d = json.load(f)
            per_kernel = None
            # round 4 added defaulted template arguments (KC, SB, POS, SAT) to k_tile_pack's name;
            # round 6 made POS an int (0 = the build, 2 = the round-6 probe pack)
            norm = lambda x: (x.replace(", 0, 20, false, false>", ">").replace(", 0, 20, 0, false>", ">")
                              .replace(", 0, 20, false>", ">").replace(", 0, 20, 0>", ">"))
            for kname, kv in d.get("kernels", {}).items():
                if kernel and norm(kernel) in norm(kname):
                    per_kernel = kv["read_bytes"] + kv["write_bytes"]
            return per_kernel, d["per_launch_bytes"], "profiles/%s/%s" % (rnd, name)
        except (OSError, ValueError, KeyError):
            continue
    return None, None, None


def vp(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else None


def log(*a):
    print(*a, file=sys.stderr, flush=True)


class Ctx:
    def __init__(self, args):
        self.world = int(os.environ.get("WORLD_SIZE", "1"))
        self.rank = int(os.environ.get("RANK", "0"))
        self.local = int(os.environ.get("LOCAL_RANK", "0"))
        self.local_world = int(os.environ.get("LOCAL_WORLD_SIZE", str(self.world)))
        # Rehearsal knobs for the N>1 path on a one-GPU box: VBF_SHARE_DEVICE=1 puts every rank
        # on cuda:0, VBF_DIST_BACKEND=gloo replaces RCCL (which refuses two ranks on one GPU).
        # The driver's multi-GPU runs set neither: one rank per GPU over RCCL.
        self.shared_device = os.environ.get("VBF_SHARE_DEVICE") == "1"
        if self.shared_device:
            self.local = 0
        self.backend = os.environ.get("VBF_DIST_BACKEND", "nccl")
        ndev = torch.cuda.device_count()
        if not self.shared_device and self.local_world > ndev:
            raise SystemExit("bench.py: %d ranks on this node but only %d visible GPUs (one rank per GPU)"
                             % (self.local_world, ndev))
        torch.cuda.set_device(self.local)
        self.dev = torch.device("cuda", self.local)
        # VBF_FORCE_PG=1: join a process group even alone, so a one-GPU box exercises the RCCL
        # calls of the N > 1 path (init, all_gather_object, all_reduce, barrier) for real
        self.pg = self.world > 1 or os.environ.get("VBF_FORCE_PG") == "1"
        if self.pg:
            if self.backend == "nccl":
                dist.init_process_group("nccl", device_id=self.dev)
            else:
                dist.init_process_group(self.backend)
            assert dist.get_world_size() == self.world, (dist.get_world_size(), self.world)
        self.stream = torch.cuda.current_stream(self.dev)
        self.sp = ctypes.c_void_p(self.stream.cuda_stream)
        self.topology = self._topology()

    def _device_info(self):
        p = torch.cuda.get_device_properties(self.dev)
        pci = "%04x:%02x:%02x" % (getattr(p, "pci_domain_id", 0), getattr(p, "pci_bus_id", 0),
                                  getattr(p, "pci_device_id", 0))
        return {"rank": self.rank, "local_rank": self.local, "device": self.local, "pci": pci,
                "name": p.name, "arch": getattr(p, "gcnArchName", ""), "host": socket.gethostname()}

    def _topology(self):
        """Every rank's device; with one rank per GPU no two ranks may share a card."""
        mine = self._device_info()
        if not self.pg:
            return {"world_size": 1, "backend": None, "ranks": [mine]}
        allr = [None] * self.world
        dist.all_gather_object(allr, mine)
        seen = {}
        for r in allr:
            key = (r["host"], r["pci"])
            if key in seen and not self.shared_device:
                raise SystemExit("bench.py: ranks %d and %d share GPU %s on %s" % (seen[key], r["rank"], r["pci"],
                                                                                  r["host"]))
            seen[key] = r["rank"]
        topo = {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": allr,
                "shared_device_rehearsal": self.shared_device}
        if self.backend == "nccl":
            try:
                topo["rccl_version"] = ".".join(str(x) for x in torch.cuda.nccl.version())
            except Exception:  # noqa: BLE001 -- informational only
                pass
        return topo

    def barrier(self):
        if self.pg:
            dist.barrier()

    def _reduce(self, x, op):
        if not self.pg:
            return x
        t = torch.tensor([x], dtype=torch.float64, device=self.dev if self.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=op)
        return float(t.item())

    def max_over_ranks(self, x):
        return self._reduce(x, dist.ReduceOp.MAX)

    def sum_over_ranks(self, x):
        return self._reduce(x, dist.ReduceOp.SUM)

    def gather(self, obj):
        """Every rank's `obj`, in rank order (on every rank)."""
        if not self.pg:
            return [obj]
        out = [None] * self.world
        dist.all_gather_object(out, obj)
        return out


def build_strategy(args):
    """The build strategy flags of one timed step: a fresh filter (new + build) unless
    --separate-zero asks for the zero fill as its own kernel."""
    from velarixdb_amd._lib import VBF_BUILD_FRESH
    return args.strategy if args.separate_zero else args.strategy | VBF_BUILD_FRESH


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
    ctx.rank_wall = t1 - t0
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


def host_cpu_info():
    """The host this rank runs on: model, the machine's logical CPUs, and the CPUs this process
    may actually use (affinity mask and cgroup quota; on the GPU box a one-GPU lease is a share of
    a larger machine)."""
    model = ""
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    logical = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        affinity = logical
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            if q != "max":
                quota = max(1, int(int(q) / int(per)))
    except (OSError, ValueError):
        pass
    usable = min(affinity, quota) if quota else affinity
    return {"model": model, "logical_cpus": logical, "affinity_cpus": affinity, "cgroup_cpu_quota": quota,
            "usable_cores": usable}


def cpu_baseline(keys_host, offsets_host, stride, n_sample, m, k, sample_desc, threads=1, lp=1):
    """The oracle (a port of bf.rs:126-128 -> :84-92) on this node's host cores."""
    import oracle
    from velarixdb_amd.keys import HostBatch
    words = np.zeros((m + 31) // 32, np.uint32)
    b = HostBatch(keys_host, offsets_host, stride, n_sample, lp)
    t0 = time.perf_counter()
    oracle.build_words(b, m, k, words=words, threads=threads)
    dt = time.perf_counter() - t0
    return {"value": n_sample / dt, "unit": "keys/s", "cores": threads, "kind": "port",
            "sample": sample_desc, "seconds": round(dt, 3)}


# ---------------------------------------------------------------------------------------
def bench_fixed(ctx, args):
    """Configs 2 / 4: fixed 16-byte keys, 10 bits per key, one filter per rank.

    Config 2 (the N=1 default): 100M keys, m = 1e9, seed 0x5EED0001.  Config 4 (the N>1 default):
    rank r builds SSTable shard r -- 50M keys, m = 5e8, seed 0x5EED0040 + r -- as one merged
    table's filter of a compaction (compactors/sized.rs:170-200, filter at :192-193)."""
    L = args.key_bytes
    lp = 0 if args.raw_keys else 1
    w = rank_workload(args, ctx.rank)
    n, m, k, seed = w["keys"], w["m"], w["k"], w["seed"]
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", seed, 0, n, L, vp(keys), ctx.sp)
    nwords = (m + 31) // 32
    words = torch.empty(nwords, dtype=torch.int32, device=ctx.dev)

    def step(evs):
        # BloomFilter::new (BitVec::from_elem(m, false), bf.rs:71) + build_filter_from_entries:
        # VBF_BUILD_FRESH writes every word of the filter (zeros included) in the build itself
        if args.separate_zero:
            words.zero_()
        if evs is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ctx.stream)
        call("vbf_build_dev_ex", vp(keys), None, L, n, lp, m, k, vp(words), build_strategy(args), ctx.sp)
        if evs is not None:
            b.record(ctx.stream)
            evs.append((a, b))

    wall, kms, phases = timed_steps(ctx, step, args.steps, args.warmup)
    rank_wall = ctx.rank_wall

    # post-timing checks on the last build: every key present; fill ratio
    cnt = torch.zeros(1, dtype=torch.int64, device=ctx.dev)
    call("vbf_probe_count_dev", vp(keys), None, L, n, lp, m, k, vp(words), vp(cnt), ctx.sp)
    pop = torch.zeros(1, dtype=torch.int64, device=ctx.dev)
    call("vbf_popcount_dev", vp(words), nwords, vp(pop), ctx.sp)
    torch.cuda.synchronize()
    assert int(cnt.item()) == n, "false negatives: %d of %d keys found" % (cnt.item(), n)
    sweep = time_probe_strategies(ctx, lambda st: call("vbf_probe_count_dev_ex", vp(keys), None, L, n, lp, m, k,
                                                       vp(words), vp(cnt), st, ctx.sp))

    total_keys = ctx.sum_over_ranks(n) * args.steps
    value = total_keys / wall
    kavg = float(np.mean(kms)) / 1e3
    bytes_per_key = L + m / (8.0 * n)
    ph = phase_report(phases, args.steps)
    # the contract's roofline: algorithmic bytes of one build / the dominant kernel's mean launch
    dom = max(ph, key=lambda q: ph[q]["ms_per_launch"] * ph[q]["launches"]) if ph else None
    dom_s = ph[dom]["ms_per_launch"] / 1e3 if dom else kavg
    achieved = n * bytes_per_key / dom_s / 1e9
    # the contract's traffic: HBM bytes of one launch of the dominant kernel (like `achieved`);
    # the whole build's bytes beside it
    rp = ROCPROF.get((L, k), (None, None)) if lp else (None, None)
    dom_kernel = (rp[0] or {}).get(dom)
    traffic_file = {10: "traffic_config2.json", 19: "traffic_config2_k19.json"}.get(k)
    traffic, traffic_build, traffic_src = (pmc_traffic(traffic_file, dom_kernel)
                                           if (n, L, lp) == (100_000_000, 16, 1) and traffic_file and args.strategy != 1
                                           else (None, None, None))
    per_rank = ctx.gather({"rank": ctx.rank, "device": ctx.local, "keys": n, "seed": seed,
                           "keys_per_s": n * args.steps / rank_wall, "ms_per_step": rank_wall / args.steps * 1e3,
                           "fill_ratio": int(pop.item()) / m})
    cfg_name = ("config4: %d independent SSTable shards x %dM x %dB keys, one per GPU (compaction fan-in), "
                "%d bits/key (m=%d, k=%d per shard)" % (ctx.world, n // 10**6, L, args.bits_per_key, m, k)
                if args.config == 4 else
                "config2: %dM x %dB keys%s%s, %d bits/key (m=%d, k=%d)" % (
                    n // 10**6, L, "" if ctx.world == 1 else " per GPU",
                    " hashed without the length prefix" if not lp else "", args.bits_per_key, m, k))
    # the SQ pass of the same build shape (config 2's 100M x 16 B keys at k = 10 or 19)
    sq = pmc_sq(SQ_FILES[k], 100_000_000) if (n, L, lp) == (100_000_000, 16, 1) and k in SQ_FILES else None
    res = {
        "metric": "Bloom build keys/s (device-resident keys, bit-exact SipHash-1-3 filter)",
        "value": value, "unit": "keys/s", "n_gpus": ctx.world, "steps": args.steps,
        "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True,
        "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "key_gib_per_s": value * L / 2**30,
        "config": {"workload": cfg_name, "baseline_config": args.config,
                   "n_keys_per_gpu": n, "key_bytes": L, "m_bits": m, "k": k, "len_prefix": bool(lp),
                   "parallelism": "independent shards x%d" % ctx.world},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_build": traffic_build,
                     "traffic_source": traffic_src, "kernel": dom, "kernel_ms": dom_s * 1e3,
                     "build_ms": kavg * 1e3, "build_frac": n * bytes_per_key / kavg / 1e9 / HBM_PEAK_GBS,
                     "rocprof_kernels": rp[0],
                     "rocprof_summary": rp[1],
                     "valu_frac_est": (n * sq["valu_lane_instr_per_key"] / dom_s / VALU_PEAK_LANE_OPS
                                       if sq else None),
                     "sq_counters": sq,
                     "algorithmic_bytes_per_key": bytes_per_key,
                     "siprounds_per_key": (L + 8) // 8 + 5 * k,
                     "phases": ph},
        "fill_ratio": int(pop.item()) / m,
        "positive_sweep_ms": sweep,
        "ranks": per_rank,
        "topology": ctx.topology,
    }
    if ctx.world == 1 and ctx.rank == 0 and not args.no_cpu_baseline:
        ns = args.cpu_sample
        host = keys[: ns * L].cpu().numpy()
        info = host_cpu_info()
        res["host_cpu"] = info
        res["cpu_baseline"] = cpu_baseline(host, None, L, ns, m, k,
                                           "first %d of the %d keys, same m=%d/k=%d, 1 thread, ref-faithful "
                                           "(full SipHash per seed, u64 %%, serial like bf.rs:127)" % (ns, n, m, k), lp=lp)
        t = args.cpu_opt_threads or info["usable_cores"]
        if t:
            res["cpu_opt"] = cpu_baseline(host, None, L, ns, m, k,
                                          "same sample, prefix-shared hashing, %d threads = every core this process "
                                          "may use (%s; %d logical CPUs on the machine)" % (
                                              t, info["model"] or "unknown CPU", info["logical_cpus"]),
                                          threads=t, lp=lp)
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
        if args.separate_zero:
            words.zero_()
        if evs is not None:
            a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            a.record(ctx.stream)
        call("vbf_build_dev_ex", vp(keys), vp(off), 0, n, 1, m, k, vp(words), build_strategy(args), ctx.sp)
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
    bpk = mean_len + 8 + m / (8.0 * n)  # key bytes + their u64 offset + the filter's bytes
    ph = phase_report(phases, args.steps)
    # as config 2: algorithmic bytes of one build / the dominant kernel's mean launch
    dom = max(ph, key=lambda q: ph[q]["ms_per_launch"] * ph[q]["launches"]) if ph else None
    dom_s = ph[dom]["ms_per_launch"] / 1e3 if dom else kavg
    achieved = n * bpk / dom_s / 1e9
    traffic, traffic_build, traffic_src = (pmc_traffic("traffic_config3.json", "k_tile_pack<-1")
                                           if n == 100_000_000 and k == 10 and args.strategy != 1
                                           else (None, None, None))
    return {
        "metric": "Bloom build keys/s (device-resident variable-length keys)", "value": value,
        "unit": "keys/s", "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic",
        "key_gib_per_s": value * mean_len / 2**30,
        "config": {"workload": "config3: %dM var-length keys (Zipf 8..128 B, mean %.1f B), %d bits/key (m=%d, k=%d) + %dM negative probes"
                   % (n // 10**6, mean_len, args.bits_per_key, m, k, nn // 10**6)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_build": traffic_build,
                     "traffic_source": traffic_src, "kernel": dom, "kernel_ms": dom_s * 1e3,
                     "build_ms": kavg * 1e3, "build_frac": n * bpk / kavg / 1e9 / HBM_PEAK_GBS,
                     "algorithmic_bytes_per_key": bpk, "phases": ph},
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

    # the full positive sweep (contains() of every key, bf.rs:95-105): one untimed call (the AUTO
    # strategy's hit-rate sample, workspace allocation), then `reps` timed calls with the library's
    # per-phase hipEvents; every call must find all N keys.  Also timed: the round-3 pipeline
    # (VBF_PROBE_PU=0, read per call) for the A/B record.
    from velarixdb_amd._lib import lib, profile_read

    def sweep_once():
        cnt.zero_()
        call("vbf_probe_count_dev", vp(keys), None, L, n, 1, m, k, vp(buf), vp(cnt), ctx.sp)

    def timed_sweeps(reps=3):
        sweep_once()
        torch.cuda.synchronize()
        ctx.barrier()
        lib.vbf_profile_enable(1)
        profile_read()
        t0 = time.perf_counter()
        for _ in range(reps):
            sweep_once()
        torch.cuda.synchronize()
        dt = ctx.max_over_ranks((time.perf_counter() - t0) / reps)
        lib.vbf_profile_enable(0)
        hits = int(ctx.sum_over_ranks(int(cnt.item())))
        assert hits == N, "positive sweep found %d of %d" % (hits, N)
        return dt, phase_report(profile_read(), reps)

    sweep, sweep_phases = timed_sweeps()
    sweep_r3 = None
    if args.probe_ab:
        os.environ["VBF_PROBE_PU"] = "0"
        try:
            sweep_r3, _ = timed_sweeps()
        finally:
            os.environ.pop("VBF_PROBE_PU", None)
    nn = args.neg_keys
    nk = torch.empty(nn * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", wl.SEED_CFG5 ^ 0xFF, N + ctx.rank * nn, nn, L, vp(nk), ctx.sp)
    cnt.zero_()
    call("vbf_probe_count_dev", vp(nk), None, L, nn, 1, m, k, vp(buf), vp(cnt), ctx.sp)
    torch.cuda.synchronize()
    fp = ctx.sum_over_ranks(int(cnt.item()))
    value = N * args.steps / wall
    # as config 2: algorithmic bytes (key bytes + this rank's share of the filter write) over the
    # dominant kernel's mean launch; the build runs in chunks, so per launch = the chunk's keys
    ph = phase_report(phases, args.steps)
    bpk = L + m / (8.0 * N)
    dom = max(ph, key=lambda q: ph[q]["ms_per_launch"] * ph[q]["launches"]) if ph else None
    roofline = None
    if dom:
        per_step = max(1.0, ph[dom]["launches"] / args.steps)
        achieved = n / per_step * bpk / (ph[dom]["ms_per_launch"] / 1e3) / 1e9
        traffic, traffic_build, traffic_src = (pmc_traffic("traffic_config5.json", "k_tile_pack<32, true, 4, false")
                                               if N == 1_000_000_000 and ctx.world == 1 and args.strategy != 1
                                               else (None, None, None))
        roofline = {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": achieved / HBM_PEAK_GBS, "traffic": traffic, "traffic_per_chunk": traffic_build,
                    "traffic_source": traffic_src, "kernel": dom, "kernel_ms": ph[dom]["ms_per_launch"],
                    "launches_per_step": per_step, "algorithmic_bytes_per_key": bpk, "phases": ph}
    return {
        "metric": "Bloom build keys/s (1B-key single filter across GPUs)", "value": value,
        "unit": "keys/s", "n_gpus": ctx.world, "steps": args.steps, "warmup": args.warmup,
        "ms_per_step": wall / args.steps * 1e3, "higher_is_better": True, "scaling": "strong",
        "vs_baseline": None, "dtype": "u64", "data": "synthetic", "key_gib_per_s": value * L / 2**30,
        "config": {"workload": "config5: %d x 32B keys, 15 bits/key -> m=%d (u32-saturated), k=%d; OR all-reduce over %d ranks" % (N, m, k, ctx.world)},
        "build_kernel_ms": float(np.mean(kms)), "roofline": roofline, "probe_sweep_keys_per_s": N / sweep,
        "probe_sweep_ms": sweep * 1e3, "probe_sweep_phases": sweep_phases,
        "probe_sweep_ms_round3_pipeline": None if sweep_r3 is None else sweep_r3 * 1e3,
        "negatives": {"n": nn * ctx.world, "false_positives": fp, "fpr": fp / (nn * ctx.world)},
    }


def bench_e2e(ctx, args):
    """Keys in host memory (memtable / compaction output): vbf_filter_set_host end to end.

    One step = BloomFilter::new (bf.rs:62-81, zeroed bits in HBM) + build_filter_from_entries over
    the host keys (H2D in chunks overlapped with the kernels) + the finished words copied into
    the caller's storage (the Rust BitVec the SST is written from).  The caller's storage is
    allocated once and reused, as a long-lived writer's buffer would be; --e2e-fresh-out copies
    into a fresh array every step (first-touch page faults included)."""
    n, L = args.keys, 16
    p = wl.fpr_for_bits_per_key(10)
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    call("vbf_gen_fixed_dev", wl.SEED_CFG2, 0, n, L, vp(keys), ctx.sp)
    host = keys.cpu().numpy()
    del keys
    from velarixdb_amd.keys import HostBatch
    hb = HostBatch(host, None, L, n, 1)
    out = None
    times, phases = [], []
    for i in range(args.warmup + args.steps):
        t0 = time.perf_counter()
        bf = vbf.BloomFilter(p, n, device=ctx.local)
        t1 = time.perf_counter()
        bf.set_batch(hb)
        t2 = time.perf_counter()
        if out is None or args.e2e_fresh_out:
            out = np.empty(bf.num_words(), dtype=np.uint32)
            if not args.e2e_fresh_out:
                out.fill(0)  # the caller's storage exists before the build (BitVec::from_elem)
                t2 = time.perf_counter()
        w = bf.words(out=out)  # D2H of the finished filter (written back with the SST)
        t3 = time.perf_counter()
        if i >= args.warmup:
            times.append(t3 - t0)
            phases.append((t1 - t0, t2 - t1, t3 - t2))
        del bf
    t = float(np.median(times))
    ph = np.median(np.array(phases), axis=0) * 1e3
    link = (n * L + 4 * w.size) / 57e9  # measured pageable H2D/D2H rate of the box
    return {"metric": "Bloom build keys/s end-to-end (host keys: H2D + build + D2H)", "value": n / t,
            "unit": "keys/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": t * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "u64", "data": "synthetic",
            "config": {"workload": "config2 e2e %dM x 16B, filter %d words, %s output storage" % (
                n // 10**6, w.size, "fresh" if args.e2e_fresh_out else "caller-owned, reused")},
            "phases_ms": {"new": ph[0], "set_host_keys": ph[1], "words_to_host": ph[2]},
            "link_floor_ms": link * 1e3}


def bench_fanout(ctx, args):
    """The compaction loop of compactors/sized.rs:170-200 as the patched bf.rs runs it
    (INTEGRATION.md): per bucket the merged table's keys are materialised on the CPU (here: copied
    into a freshly allocated packed buffer, the merge's output), then BloomFilter::new(fpr, n) and
    build_filter_from_entries.  `sync`: the build is vbf_filter_set_host on a fixed device (returns
    with the bits done); `async`: VBF_DEVICE_AUTO placement and vbf_filter_set_host_async with the
    release callback (returns at once, so the next bucket's materialisation overlaps the GPU
    build).  Each mode ends when every filter's words are fetched (the SST writes) and the words
    of both modes are compared.  One GPU here: the overlap is host work vs one GPU's H2D + build;
    with 8 GPUs, AUTO puts consecutive buckets on different GPUs."""
    B, n, L = args.buckets, args.keys, 16
    p = wl.fpr_for_bits_per_key(10)
    from velarixdb_amd.keys import HostBatch
    srcs = []
    keys = torch.empty(n * L, dtype=torch.uint8, device=ctx.dev)
    for b in range(B):
        call("vbf_gen_fixed_dev", wl.SEED_CFG4 + b, 0, n, L, vp(keys), ctx.sp)
        srcs.append(keys.cpu().numpy())
    del keys

    def run(mode):
        t0 = time.perf_counter()
        filters, merge_s = [], 0.0
        for b in range(B):
            m0 = time.perf_counter()
            if args.fanout_reuse:
                buf = srcs[b]  # no materialisation: the builds alone
            else:
                buf = np.empty_like(srcs[b])
                np.copyto(buf, srcs[b])  # the merged table's keys, packed
            merge_s += time.perf_counter() - m0
            hb = HostBatch(buf, None, L, n, 1)
            if mode == "sync":
                f = vbf.BloomFilter(p, n, device=ctx.local)
                f.set_batch(hb)
            else:
                f = vbf.BloomFilter(p, n, device="host")  # new() keeps a fresh filter on the host
                f.migrate("auto")  # build_filter_from_entries: the library places it (no bits copied)
                f.set_many_async(hb, zero_copy=True)
            filters.append(f)
        t_loop = time.perf_counter() - t0
        words = [f.words() for f in filters]  # the SST writes wait for their filter
        return time.perf_counter() - t0, t_loop, merge_s, words

    for _ in range(args.warmup):
        run("sync")
        run("async")
    res = {}
    for mode in ("sync", "async"):
        ts = [run(mode) for _ in range(args.steps)]
        i = int(np.argsort([t[0] for t in ts])[len(ts) // 2])
        res[mode] = {"total_ms": ts[i][0] * 1e3, "loop_ms": ts[i][1] * 1e3, "materialise_ms": ts[i][2] * 1e3,
                     "keys_per_s": B * n / ts[i][0], "words": ts[i][3]}
    same = all(np.array_equal(a, b) for a, b in zip(res["sync"]["words"], res["async"]["words"]))
    for mode in res:
        del res[mode]["words"]
    assert same, "async builds differ from the synchronous ones"
    return {"metric": "compaction loop keys/s (materialise + new + build per bucket, then the SST writes)",
            "value": res["async"]["keys_per_s"], "unit": "keys/s", "n_gpus": 1, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": res["async"]["total_ms"], "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "%d buckets x %dM x 16B host keys, 10 bits/key" % (B, n // 10**6)},
            "modes": res, "async_words_equal_sync": same,
            "speedup": res["sync"]["total_ms"] / res["async"]["total_ms"]}


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

    wall, _, phases = timed_steps(ctx, step, args.steps, args.warmup)
    hits = int(out.view(n, S).any(dim=1).sum().item())
    return {"metric": "multi-SST probe keys/s (each key tested against 8 filters, device-resident)",
            "value": ctx.sum_over_ranks(n) * args.steps / wall, "unit": "keys/s", "n_gpus": ctx.world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": wall / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "%dM x 16B keys vs %d filters of 10M keys (m=1e8, k=10); %d keys hit some SST"
                       % (n // 10**6, S, hits)},
            "probes_per_s": ctx.sum_over_ranks(n) * S * args.steps / wall,
            "phases": phase_report(phases, args.steps)}


def bench_memtable(ctx, args):
    """Single-key latency of the memtable's filter calls (mem.rs:209-211 contains + set per put,
    :224 contains per get) through the C ABI from a plain C host (examples/memtable_latency.c),
    host-resident vs device-resident; the tool also checks both residencies end bit-identical."""
    tool = os.path.join(ROOT, "examples", "memtable_latency")
    out = subprocess.run([tool, str(args.keys or 200_000), "2000"], capture_output=True, text=True, timeout=600)
    if out.returncode != 0:
        raise SystemExit("memtable_latency failed: " + out.stderr[-2000:])
    r = json.loads(out.stdout.strip().splitlines()[-1])
    return {"metric": "memtable filter single-key latency (contains + set per put, contains per get)",
            "value": r["host"]["put_us"]["mean"], "unit": "us/put", "n_gpus": 1, "steps": r["host"]["keys"],
            "warmup": 0, "higher_is_better": False, "dtype": "u64", "data": "synthetic",
            "config": {"workload": "memtable filter m=%d k=%d (51 200-byte write buffer / 100 entries, p=1e-4)"
                       % (r["m"], r["k"])},
            "detail": r}


def rank_workload(args, rank):
    """(config, keys, m, k, seed) of `rank`'s build in the fixed-key configs (2 and 4)."""
    n = args.keys or (100_000_000 if args.config == 2 else 50_000_000)
    p = wl.fpr_for_bits_per_key(args.bits_per_key)
    m = vbf.num_bits(n, p)
    seed = (wl.SEED_CFG4 + rank) if args.config == 4 else (wl.SEED_CFG2 + 0x100 * rank)
    return {"config": args.config, "keys": n, "m": m, "k": vbf.num_hash_functions(m, n), "seed": seed}


def plan_only(args, world):
    """The launch without the work: every rank joins the process group (gloo, CPU only) and
    reports its workload; rank 0 prints them.  Tests the spawn path where there is no GPU."""
    rank = int(os.environ.get("RANK", "0"))
    if world > 1:
        dist.init_process_group("gloo")
        assert dist.get_world_size() == world
    mine = dict(rank_workload(args, rank), rank=rank, local_rank=int(os.environ.get("LOCAL_RANK", "0")))
    allr = [None] * world
    if world > 1:
        dist.all_gather_object(allr, mine)
    else:
        allr = [mine]
    if rank == 0:
        print(json.dumps({"plan_only": True, "world_size": world, "n_gpus": args.gpus, "ranks": allr}), flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    args = make_parser().parse_args()
    mode, world = launch_plan(args.gpus, os.environ)
    assert mode == "run", "maybe_spawn_ranks() handles --gpus N > 1 without a launcher"
    args.gpus = world
    if args.config is None:
        args.config = 2 if world == 1 else 4
    if args.plan_only:
        return plan_only(args, world)
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
    elif args.memtable:
        res = bench_memtable(ctx, args)
    elif args.fanout:
        args.keys = args.keys or 12_500_000
        res = bench_fanout(ctx, args)
    else:
        args.keys = args.keys or (100_000_000 if args.config == 2 else 50_000_000)
        res = bench_fixed(ctx, args)
    if ctx.rank == 0:
        print(json.dumps(res), flush=True)
    if ctx.pg:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
