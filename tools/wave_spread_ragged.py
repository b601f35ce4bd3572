#!/usr/bin/env python3
"""Per-wave timeline of the ragged kernels (round 6):
does the static schedule -- one byte-balanced range per wave, or per wave and
chunk -- leave the GPU partly idle at the end of a launch, as it did for the
fixed kernel before its LDS work counter (tools/wave_spread.py)?

    LSBM_LIB_PATH=build/r6/diag/liblsbm_crc32c.so python tools/wave_spread_ragged.py [entry ...]

Needs a -DLSBM_DIAG_STAMPS build (tools/build_variant.sh NAME '1i #define
LSBM_DIAG_STAMPS' crc32c_units.h): every wave of the units, stream and fixed
kernels stamps its start, its first data and its end (s_memrealtime, 100 MHz).
Entries:
  config4     10M Zipf blocks (117 GiB), lsbm_crc32c_batch_dev -> crc32c_stream_kernel<32,Out,offsets>
  sst_verify  1M x 4,118-B SSTable blocks, lsbm_sst_verify_dev  -> crc32c_units_kernel<40,SstVerify>
  sst_crcs    the same image, lsbm_sst_trailer_crcs_dev         -> crc32c_units_kernel<40,SstCrc>
  sst_seal    the same image, lsbm_sst_seal_dev                 -> crc32c_units_kernel<40,SstCrc> + trailers
  fixed4k     config 2, for comparison                          -> crc32c_fixed_kernel<false,32>
One JSON line per entry: the launch span, the waves' durations (mean, CV),
when the first wave finished (fraction of the span: the GPU is partly idle
from there on) and the spread of the waves' ends.
"""
import ctypes
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)

from bench_configs import zipf_lengths  # noqa: E402


def timeline(st, alg_bytes):
    nw = int(np.count_nonzero(st[2]))
    start, first, end = (st[k][:nw].astype(np.int64) for k in range(3))
    t0 = start.min()
    span = (end.max() - t0) / 100.0  # us
    dur = (end - start) / 100.0
    endr = (end - t0) / 100.0
    setup = (first - start) / 100.0
    xcc = st[3][:nw].astype(np.int64)
    wpw = int(os.environ.get("LSBM_WAVES_PER_WG", "16"))
    wg = np.arange(nw) // wpw
    ngw = nw // wpw
    wg_end = np.array([endr[wg == g].max() for g in range(ngw)])
    wg_in = np.array([endr[wg == g].max() - endr[wg == g].min() for g in range(ngw)])
    by_xcc = {int(x): [round(float(endr[xcc == x].mean()), 1), round(float(dur[xcc == x].mean()), 1)]
              for x in np.unique(xcc)}
    extra = {"by_xcc_mean_end_dur_us": by_xcc,
             "wg_end_p0_p50_p100_us": [round(float(x), 1) for x in np.percentile(wg_end, [0, 50, 100])],
             "within_wg_end_spread_mean_us": round(float(wg_in.mean()), 1)}
    return {"waves": nw, **extra, "span_us": round(float(span), 1),
            "GBps_span": round(alg_bytes / (span / 1e6) / 1e9, 1),
            "pct_hbm_span": round(100 * alg_bytes / (span / 1e6) / 8e12, 2),
            "start_spread_us": round(float((start - t0).max() / 100.0), 1),
            "setup_us_mean": round(float(setup.mean()), 2),
            "dur_mean_us": round(float(dur.mean()), 1),
            "dur_cv": round(float(dur.std() / dur.mean()), 4),
            "dur_min_max_us": [round(float(dur.min()), 1), round(float(dur.max()), 1)],
            "end_p0_p10_p50_p90_p100_us": [round(float(x), 1) for x in np.percentile(endr, [0, 10, 50, 90, 100])],
            "first_end_frac": round(float(endr.min() / span), 4),
            "tail_frac": round(float((span - endr.min()) / span), 4)}


def run(entry, lb, stamps_fn, launch, alg, reps=3):
    import torch
    st = np.zeros((4, 65536), dtype=np.uint64)
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < 0.3:  # clock spin-up
        launch()
        torch.cuda.synchronize()
    for r in range(reps):
        launch()
        torch.cuda.synchronize()
        st[:] = 0
        assert stamps_fn(st.ctypes.data, 4 * 65536) == 0
        rec = {"entry": entry, "rep": r, "algorithmic_bytes": int(alg)}
        rec.update(timeline(st, alg))
        print(json.dumps(rec), flush=True)
        dump = os.environ.get("LSBM_STAMPS_DUMP")  # a directory: the raw stamps per entry and rep
        if dump:
            os.makedirs(dump, exist_ok=True)
            np.save(os.path.join(dump, f"{entry}_{r}.npy"), st[:, :rec["waves"]])


def main():
    import torch
    from lsbm_amd import engine, table
    from lsbm_amd._lib import lib
    torch.cuda.set_device(0)
    engine.init(0)
    lb = lib()
    fns = []
    for name in ("lsbm_diag_stamps", "lsbm_diag_stamps_stream"):
        f = getattr(lb, name, None)  # (a variant may stamp one kernel source only)
        if f is not None:
            f.argtypes = [ctypes.c_void_p, ctypes.c_int]
        fns.append(f)
    units, stream = fns
    entries = sys.argv[1:] or ["config4", "sst_verify", "sst_crcs", "sst_seal", "fixed4k"]
    s = torch.cuda.current_stream()
    if "fixed4k" in entries:
        n, L = 1 << 20, 4096
        d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
        engine.fill_splitmix64(d, 0x5EED0000)
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        run("fixed4k", lb, units, lambda: engine.crc32c_fixed(d, L, L, n, out=out, stream=s), n * L)
        del d, out
    if any(e.startswith("sst") for e in entries):
        n, L = 1 << 20, 4118
        offs = np.arange(n + 1, dtype=np.int64) * (L + 5)
        d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
        engine.fill_splitmix64(d, 0x5EED0005)
        handles = torch.from_numpy(np.stack([offs[:-1], np.full(n, L, dtype=np.int64)], 1)
                                   .reshape(-1).copy()).to("cuda")
        types = torch.zeros(n, dtype=torch.uint8, device="cuda")
        tc = torch.empty(n, dtype=torch.int32, device="cuda")
        nb = torch.zeros(1, dtype=torch.int32, device="cuda")
        alg = n * (L + 1)
        if "sst_seal" in entries:
            run("sst_seal", lb, units, lambda: table.seal_blocks(d, handles, types, stream=s), alg)
        if "sst_verify" in entries:
            run("sst_verify", lb, units, lambda: table.verify_blocks(d, handles, stream=s), alg)
        if "sst_crcs" in entries:
            run("sst_crcs", lb, units, lambda: table.trailer_crcs(d, handles, types, stream=s, out=tc, nbad=nb), alg)
        del d, handles, types, tc
    if "config4" in entries:
        n = 10_000_000
        lens = zipf_lengths(n)
        offs = np.zeros(n + 1, dtype=np.int64)
        offs[1:] = np.cumsum(lens)
        offs += 5
        d = torch.empty(int(offs[-1]) + 16, dtype=torch.uint8, device="cuda")
        engine.fill_splitmix64(d, 0x5EED0003)
        do = torch.from_numpy(offs).to("cuda")
        out = torch.empty(n, dtype=torch.int32, device="cuda")
        run("config4", lb, stream, lambda: engine.crc32c_batch(d, do, out=out, stream=s), int(lens.sum()))
        del d, do, out
    torch.cuda.empty_cache()


if __name__ == "__main__":
    main()
