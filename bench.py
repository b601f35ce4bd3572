#!/usr/bin/env python3
"""Headline benchmark: CRC32C GiB/s over device-resident 4 KiB SSTable blocks.

Workload (BASELINE.json configs[1]): 1,048,576 blocks x
4096 B = 4 GiB per GPU, stride 4096, resident in HBM before timing starts.
The bytes: one dataset, block i = bytes [4096 i, 4096 (i + 1)) of the
splitmix64 stream 0x5EED0000 (tests/golden/splitmix.py), generated on the
device; rank r of N holds global blocks [r n, (r + 1) n).  One
*step* = one lsbm_crc32c_fixed_dev call over the whole batch (crc32c::Value
of every block, util/crc32c.cc:286-329): one launch for the 1M-block config,
back-to-back launches of 1M blocks for a 10M-block shard.

    python bench.py [--gpus N] [--steps K] [--warmup W]

With N > 1 it runs one process per GPU under torch.distributed.run: when
WORLD_SIZE is unset, bench.py starts `python -m torch.distributed.run
--nproc-per-node N ... bench.py` itself as a child process (before any GPU
call) and exits with its return code; a WORLD_SIZE that differs from --gpus is
an error.  Each rank checksums its own shard of 10M x 4 KiB blocks (BASELINE.json configs[4]:
the 80M-block dataset over 8 GPUs in contiguous ranges, blocks [10M r, 10M (r + 1)) on
rank r, so any N checksums the same bytes for the same block; weak scaling, no
data-path collective: blocks are independent).  --blocks overrides the per-GPU block count.  Timing: W untimed steps, barrier + synchronize, K
steps between HIP events on the launch stream, barrier + synchronize, max over
ranks.  Rank 0 prints ONE JSON line.

Extra fields: roofline (achieved algorithmic GB/s of the dominant kernel vs the
8 TB/s HBM peak), cpu_baseline (the reference CPU CRC on the host cores, rank 0
at N=1 only, bounded sample), stream_read (the same buffer read with the CRC
kernel's own access pattern and no CRC work: the measured read ceiling),
host_staged (the same blocks checksummed from pinned host memory through
lsbm_crc32c_batch_host: the PCIe-inclusive rate, rank 0 at N=1 only), ranks
(per rank: its own elapsed time, bytes, GiB/s and kernel time per launch, its
device's PCI address and NUMA node and its CPUs' NUMA nodes; the bytes add up
to the aggregate).
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = "CRC32C GiB/s over device-resident 4 KiB SSTable blocks (1 GPU); % HBM peak"
HBM_PEAK_GBPS = 8000.0  # MI355X spec, MI355X_MICROARCH.md "Chip-level parameters"
BLOCK = 4096
NBLOCKS = 1 << 20            # configs[1]: 1M x 4 KiB on one GPU
NBLOCKS_MULTI = 10_000_000   # configs[4]: 80M x 4 KiB over 8 GPUs = 10M per GPU
SEED = 0x5EED0000


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=50)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--blocks", type=int, default=0, help=argparse.SUPPRESS)
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=12.0,
                   help="aggregate CPU-seconds for the cpu_baseline sample")
    p.add_argument("--dump-samples", default="", help=argparse.SUPPRESS)  # tests: per-rank CRCs
    p.add_argument("--spin-s", type=float, default=0.5,
                   help="seconds of untimed launches before the warm-up steps (GPU clock ramp)")
    return p.parse_args()


def usable_cores():
    """Host cores this process may run on: the affinity mask, capped by a
    cgroup CPU quota when one is set (the GPU box's CPU share)."""
    n = len(os.sched_getaffinity(0))
    quota = None
    for path, conv in (("/sys/fs/cgroup/cpu.max", lambda t: t.split()),
                       ("/sys/fs/cgroup/cpu/cpu.cfs_quota_us", lambda t: [t.strip(), None])):
        try:
            with open(path) as f:
                q = conv(f.read())
        except OSError:
            continue
        try:
            if q[0] != "max" and int(q[0]) > 0:
                period = int(q[1]) if q[1] else int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
                quota = max(1, int(q[0]) // period)
        except (OSError, ValueError, IndexError):
            pass
        break
    return (min(n, quota) if quota else n), n, quota


def launch_ranks(args):
    """--gpus N > 1 without WORLD_SIZE: run this script under
    torch.distributed.run as a CHILD process (nothing here has touched the GPU)
    and return its exit code."""
    import socket
    import subprocess
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1",
           f"--nproc-per-node={args.gpus}", "--master-addr=127.0.0.1", f"--master-port={port}",
           os.path.abspath(__file__)] + sys.argv[1:]
    return subprocess.run(cmd).returncode


def shard_range(n_total, rank, world):
    """Contiguous shard [lo, hi) of n_total independent blocks for `rank`.
    Blocks never cross ranks: the CRC of a block needs only its own bytes."""
    per = (n_total + world - 1) // world
    lo = min(n_total, rank * per)
    return lo, min(n_total, lo + per)


def timed_steps(step, steps, warmup, sync, barrier, max_reduce, mark_start=None, mark_end=None):
    """The driver's timing contract: `warmup` untimed steps, barrier +
    synchronize, `steps` timed steps, barrier + synchronize.  Returns the MAX
    over ranks of this rank's wall seconds for the timed region.  mark_start /
    mark_end bracket exactly the timed launches (device events)."""
    for _ in range(warmup):
        step()
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    if mark_start:
        mark_start()
    for _ in range(steps):
        step()
    if mark_end:
        mark_end()
    sync()
    barrier()
    sync()
    return max_reduce(time.perf_counter() - t0)


def numa_node_of_cpus(cpus):
    """The NUMA node(s) holding `cpus` (sysfs node cpulists), as a sorted list."""
    nodes = set()
    base = "/sys/devices/system/node"
    try:
        names = [d for d in os.listdir(base) if d.startswith("node") and d[4:].isdigit()]
    except OSError:
        return []
    for d in names:
        try:
            with open(os.path.join(base, d, "cpulist")) as f:
                text = f.read().strip()
        except OSError:
            continue
        for part in filter(None, text.split(",")):
            a, _, b = part.partition("-")
            lo, hi = int(a), int(b or a)
            if any(lo <= c <= hi for c in cpus):
                nodes.add(int(d[4:]))
                break
    return sorted(nodes)


def device_placement(torch, device):
    """Where rank's GPU sits: its PCI address and that device's NUMA node
    (sysfs), beside the NUMA node(s) of the CPUs this process may run on --
    the first thing to look at when one rank of a node is slow."""
    rec = {"device": device}
    try:
        p = torch.cuda.get_device_properties(device)
        rec["name"] = p.name
        dom, bus, dev = (getattr(p, k, None) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id"))
        if bus is not None:
            addr = f"{dom or 0:04x}:{bus:02x}:{dev or 0:02x}.0"
            rec["pci"] = addr
            try:
                with open(f"/sys/bus/pci/devices/{addr}/numa_node") as f:
                    rec["gpu_numa_node"] = int(f.read().strip())
            except (OSError, ValueError):
                rec["gpu_numa_node"] = None
    except Exception as e:  # (a record, not a reason to fail the bench)
        rec["error"] = str(e)
    rec["cpu_numa_nodes"] = numa_node_of_cpus(os.sched_getaffinity(0))
    return rec


def rank_record(rank, elapsed_s, nbytes, kernel_ms_per_launch, placement):
    """This rank's own line of the per-rank table (bench.py's JSON `ranks`)."""
    return dict(rank=rank, elapsed_s=round(elapsed_s, 6), bytes=int(nbytes),
                GiBps=round(nbytes / elapsed_s / 2**30, 2) if elapsed_s > 0 else None,
                kernel_ms_per_launch=None if kernel_ms_per_launch is None else round(kernel_ms_per_launch, 4),
                **placement)


def gather_ranks(dist, world, rec):
    """Every rank's record, in rank order, over the harness's process group
    (gloo by default: CPU objects, no RCCL)."""
    if world == 1:
        return [rec]
    out = [None] * world
    dist.all_gather_object(out, rec)
    return sorted(out, key=lambda r: r["rank"])


def load_traffic(workload):
    """HBM bytes per launch from a committed rocprofv3 PMC pass, if any."""
    path = os.path.join(REPO, "profiles", "traffic.json")
    try:
        with open(path) as f:
            d = json.load(f)
        if d.get("workload") == workload:
            return float(d["hbm_bytes_per_launch"])
    except (OSError, ValueError, KeyError):
        pass
    return None


def cpu_baseline(host, gpu_crcs, cpu_seconds):
    """Time the CPU CRC-32C on the host: the reference's own util/crc32c.cc
    (oracle/_ref, built from /root/reference) when present, else the oracle's
    plain-C restatement of it.  `host` is a host copy of the whole device
    batch; every block is also cross-checked against the GPU results."""
    import subprocess
    ref = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
    port = os.path.join(REPO, "oracle", "liboracle_crc32c.so")
    if os.path.exists(ref):
        lib, fn, kind = ctypes.CDLL(ref), "ref_batch_fixed_mt", "reference"
    else:
        if not os.path.exists(port):
            subprocess.run(["make", "-C", os.path.join(REPO, "oracle")], check=True,
                           stdout=subprocess.DEVNULL)
        lib, fn, kind = ctypes.CDLL(port), "oracle_batch_fixed_mt", "port"
    f = getattr(lib, fn)
    f.restype = ctypes.c_int
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_uint64, ctypes.c_uint64,
                  ctypes.c_void_p, ctypes.c_int]
    n = host.size // BLOCK
    out = np.empty(n, dtype=np.uint32)
    threads, affinity, quota = usable_cores()
    threads = min(threads, 256)
    f(host.ctypes.data, BLOCK, BLOCK, n, out.ctypes.data, threads)  # warm + cross-check
    mismatches = int(np.count_nonzero(out != gpu_crcs[:n]))
    passes, t0 = 0, time.perf_counter()
    while True:  # >= 2 passes, >= 1 s wall, ~cpu_seconds of CPU work, <= 30 s
        f(host.ctypes.data, BLOCK, BLOCK, n, out.ctypes.data, threads)
        passes += 1
        el = time.perf_counter() - t0
        if (passes >= 2 and el >= 1.0 and el * threads >= cpu_seconds) or el > 30:
            break
    gib = passes * n * BLOCK / 2**30
    # one core, bounded to ~3 s (1 thread and all threads)
    p1, t1 = 0, time.perf_counter()
    while True:
        f(host.ctypes.data, BLOCK, BLOCK, 8192, out.ctypes.data, 1)
        p1 += 1
        el1 = time.perf_counter() - t1
        if el1 >= 3.0:
            break
    # the strongest CPU CRC-32C the host has (SSE4.2 crc32, three blocks
    # interleaved), labelled "not reference" (SURVEY.md 8d): lsbm never uses it
    sse = None
    sse_path = os.path.join(REPO, "oracle", "libsse42_baseline.so")
    if not os.path.exists(sse_path):
        subprocess.run(["make", "-C", os.path.join(REPO, "oracle"), "libsse42_baseline.so"],
                       stdout=subprocess.DEVNULL)
    if os.path.exists(sse_path):
        hw = ctypes.CDLL(sse_path).sse42_batch_fixed_mt
        hw.restype = ctypes.c_int
        hw.argtypes = f.argtypes
        hw(host.ctypes.data, BLOCK, BLOCK, n, out.ctypes.data, threads)
        sse_bad = int(np.count_nonzero(out != gpu_crcs[:n]))
        ps, ts = 0, time.perf_counter()
        while True:  # >= 2 passes, <= ~3 s
            hw(host.ctypes.data, BLOCK, BLOCK, n, out.ctypes.data, threads)
            ps += 1
            els = time.perf_counter() - ts
            if ps >= 2 and els >= 1.0 or els > 3.0:
                break
        sse = {"value": round(ps * n * BLOCK / 2**30 / els, 3), "unit": "GiB/s", "cores": threads,
               "kind": "not reference (SSE4.2 crc32, 3 blocks interleaved; oracle/sse42_baseline.c)",
               "sample": f"{ps} passes x {n} x {BLOCK} B blocks, {els:.1f} s",
               "gpu_mismatches_on_sample": sse_bad}
    cpu_model = ""
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                cpu_model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"value": round(gib / el, 3), "unit": "GiB/s", "cores": threads, "kind": kind,
            "sample": f"{passes} passes x {n} x {BLOCK} B blocks (host copy of the whole "
                      f"device batch), crc32c::Value slice-by-4, {threads} pthreads = all "
                      f"usable cores (affinity {affinity}, cgroup quota {quota or 'none'}), "
                      f"{el:.1f} s wall; {cpu_model}",
            "single_thread": {"value": round(p1 * 8192 * BLOCK / 2**30 / el1, 3), "unit": "GiB/s",
                              "cores": 1, "sample": f"{p1} passes x 8192 blocks, {el1:.1f} s"},
            "gpu_mismatches_on_sample": mismatches,
            "sse42_not_reference": sse}


def host_staged(engine, data, gpu_crcs, n_blocks, reps=3):
    """PCIe-inclusive rate: blocks start in PINNED host memory,
    lsbm_crc32c_batch_host DMAs them to the GPU (hipMemcpyAsync, 64 MiB chunks
    over 3 streams overlapped with the kernel) and returns 4 B/block to the
    host.  Never the headline `value`: the north_star metric is device-resident."""
    import torch
    src = torch.empty(n_blocks * BLOCK, dtype=torch.uint8, pin_memory=True)
    src.copy_(data[:n_blocks * BLOCK])
    h = src.numpy()
    offs = np.arange(0, (n_blocks + 1) * BLOCK, BLOCK, dtype=np.uint64)
    # one untimed full pass: staging buffers, and the first DMA touch of every
    # pinned page (GPU-side mappings of host memory), as for the copy below
    engine.crc32c_batch_host(h, offs)
    t0 = time.perf_counter()
    for _ in range(reps):
        got = engine.crc32c_batch_host(h, offs)
    el = (time.perf_counter() - t0) / reps
    # the PCIe ceiling: a plain pinned H2D copy of the same bytes
    dst = torch.empty_like(src, device="cuda")
    dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        dst.copy_(src, non_blocking=True)
    torch.cuda.synchronize()
    el_copy = (time.perf_counter() - t0) / reps
    return {"GBps": round(n_blocks * BLOCK / el / 1e9, 2),
            "h2d_copy_GBps": round(n_blocks * BLOCK / el_copy / 1e9, 2),
            "GiBps": round(n_blocks * BLOCK / el / 2**30, 2),
            "sample": f"{n_blocks} x {BLOCK} B blocks from pinned host memory, {reps} passes, "
                      "host->device DMA + kernel + 4 B/block back, wall clock",
            "mismatches_vs_device_path": int(np.count_nonzero(got != gpu_crcs[:n_blocks]))}


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args)
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        print(f"error: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
        return 2
    # LSBM_BENCH_DEVICES lets a rehearsal put several ranks on fewer GPUs.
    # The shards never exchange data (north_star: "no RCCL collective"): the
    # harness's barrier and MAX of the elapsed time go over gloo on CPU
    # tensors, the code path tests/test_multirank_gpu.py runs.
    # LSBM_BENCH_BACKEND=nccl (opt-in) does them over RCCL instead.
    ndev = int(os.environ.get("LSBM_BENCH_DEVICES", "0")) or torch.cuda.device_count()
    local = local % max(1, ndev)
    torch.cuda.set_device(local)
    backend = os.environ.get("LSBM_BENCH_BACKEND", "gloo")
    if world > 1:
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)

    from lsbm_amd import engine
    engine.init(local)
    n = args.blocks or (NBLOCKS if world == 1 else NBLOCKS_MULTI)
    data = torch.empty(n * BLOCK, dtype=torch.uint8, device="cuda")
    # global blocks [lo, lo + n): the stream from byte 4096 lo, i.e. word 512 lo
    lo = rank * n
    engine.fill_splitmix64(data, SEED + lo * (BLOCK // 8))
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    stream = torch.cuda.current_stream()

    def step():
        engine.crc32c_fixed(data, BLOCK, BLOCK, n, out=out, stream=stream)

    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

    def barrier():
        if world > 1:
            dist.barrier()

    mine = {}

    def max_reduce(x):
        mine["elapsed_s"] = x  # (this rank's own time, for the per-rank table)
        t = torch.tensor([x], dtype=torch.float64, device="cuda" if backend == "nccl" else "cpu")
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        return float(t.item())

    # Untimed spin-up before the warm-up steps: after the host-side setup the
    # GPU clock has dropped, and it takes longer than a few 0.65 ms launches to
    # climb back (the same kernel measured 81-82% of HBM
    # peak right after a pause and 84-85% at steady clocks).  A compaction
    # stream keeps the GPU busy; the timed region measures that steady state.
    t_spin = time.perf_counter()
    while time.perf_counter() - t_spin < args.spin_s:
        step()
        torch.cuda.synchronize()
    t_max = timed_steps(step, args.steps, args.warmup, torch.cuda.synchronize, barrier, max_reduce,
                        mark_start=lambda: ev0.record(stream), mark_end=lambda: ev1.record(stream))
    kern_ms = ev0.elapsed_time(ev1)  # the K launches, HIP events on the launch stream

    # per-launch HIP events after the timed region (SURVEY.md 8d asks for the
    # median launch): each launch bracketed by its own pair of events
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
           for _ in range(max(3, args.steps))]
    for a, b in evs:
        a.record(stream)
        step()
        b.record(stream)
    torch.cuda.synchronize()
    per_launch_ms = sorted(a.elapsed_time(b) for a, b in evs)
    median_ms = per_launch_ms[len(per_launch_ms) // 2]

    # stream-read ceiling on the same buffer (same stream, same events)
    sink = torch.zeros(1024, dtype=torch.int32, device="cuda")
    for _ in range(3):
        engine.stream_read(data, sink, stream=stream)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(10):
        engine.stream_read(data, sink, stream=stream)
    e1.record(stream)
    torch.cuda.synchronize()
    stream_gbps = 10 * n * BLOCK / (e0.elapsed_time(e1) / 1e3) / 1e9

    # per rank: its own elapsed time, bytes and rate, and where its GPU and
    # CPUs sit (the aggregate `value` alone hides a slow rank)
    ranks = gather_ranks(dist, world, rank_record(rank, mine["elapsed_s"], n * BLOCK * args.steps,
                                                  kern_ms / args.steps, device_placement(torch, local)))

    total_bytes = n * BLOCK * world * args.steps
    value = total_bytes / t_max / 2**30
    per_launch_s = kern_ms / 1e3 / args.steps
    achieved = n * BLOCK / per_launch_s / 1e9
    workload = f"{n} x {BLOCK} B device-resident blocks per GPU, batched crc32c::Value"
    traffic = load_traffic(workload)

    if args.dump_samples:  # tests/test_multirank_gpu.py checks these against the oracle
        idx = np.unique(np.concatenate([np.arange(min(n, 64)), np.arange(max(0, n - 64), n),
                                        np.random.default_rng(rank).integers(0, n, 128)]))
        # (and every CRC of the shard at once: the XOR of all of them against
        # the oracle's CRC of the XOR of all blocks, by linearity; after timing)
        sys.path.insert(0, os.path.join(REPO, "tests"))
        from golden.xorfold import xor_fold_rows
        xb = xor_fold_rows(data.view(torch.int64).view(n, BLOCK // 8)).cpu().numpy().view(np.uint8)
        xc = xor_fold_rows(out.view(n, 1)).cpu().numpy().view(np.uint32)
        np.savez(f"{args.dump_samples}.rank{rank}.npz", gidx=lo + idx, seed=SEED, n=n,
                 crc=out.cpu().numpy().view(np.uint32)[idx], world=world, t_max=t_max,
                 xor_block=xb, xor_crc=xc)

    cpu = staged = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        gpu_crcs = out.cpu().numpy().view(np.uint32)
        staged = host_staged(engine, data, gpu_crcs, min(n, 1 << 18))
        cpu = cpu_baseline(data.cpu().numpy(), gpu_crcs, args.cpu_seconds)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": round(value, 2),
            "unit": "GiB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(t_max * 1e3 / args.steps, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "u8",
            "data": f"synthetic: one dataset, block i = bytes [4096 i, 4096 (i+1)) of the splitmix64 "
                    f"stream 0x{SEED:X}, generated on the device; rank r holds blocks [{n} r, {n} (r+1)); "
                    "resident in HBM before timing",
            "config": {"workload": workload, "blocks_per_gpu": n, "block_bytes": BLOCK,
                       "stride": BLOCK,
                       "baseline_config": "BASELINE.json configs[1]" if n == NBLOCKS and world == 1
                       else ("BASELINE.json configs[4] (10M x 4 KiB per GPU, weak scaling)"
                             if n == NBLOCKS_MULTI else "custom"),
                       "parallelism": f"{world} independent shards, no data-path collective"
                                      + (f" (timing barrier + MAX over {backend})" if world > 1 else "")},
            "pct_hbm_peak": round(100 * achieved / HBM_PEAK_GBPS, 2),
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBPS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBPS, 4),
                         "traffic": traffic,
                         "kernel": "crc32c_fixed_kernel<false,32>",
                         "algorithmic_bytes_per_launch": n * BLOCK,
                         "avg_launch_ms": round(per_launch_s * 1e3, 4),
                         "median_launch_ms": round(median_ms, 4),
                         "frac_at_median": round(n * BLOCK / (median_ms / 1e3) / 1e9 / HBM_PEAK_GBPS, 4)},
            "stream_read": {"GBps": round(stream_gbps, 1),
                            "crc_frac_of_stream_read": round(achieved / stream_gbps, 4)},
            "cpu_baseline": cpu,
            "host_staged": staged,
            "ranks": ranks,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
