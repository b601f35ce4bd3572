#!/usr/bin/env python3
"""Per-wave timeline of one fixed-kernel launch, 1M against 10M blocks
(why one launch over a 10M-block shard runs slower).

    LSBM_LIB_PATH=build/diag_stamps/liblsbm_crc32c.so LSBM_FIXED_SPLIT_BLOCKS=0 \
        python tools/wave_spread.py

Needs a -DLSBM_DIAG_STAMPS build of the library (tools/build_variant.sh diag
'1i #define LSBM_DIAG_STAMPS' crc32c_kernels.hip): every wave stamps its
start, its first data and its end with s_memrealtime (100 MHz).  Each wave
takes the same number of 8-block groups (+-1), so the spread of the waves'
durations is the spread of their rates; at the end of the launch the fastest
and the slowest wave are that fraction of the batch apart."""
import ctypes
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    import torch
    from lsbm_amd import engine
    from lsbm_amd._lib import lib
    torch.cuda.set_device(0)
    engine.init(0)
    lb = lib()
    lb.lsbm_diag_stamps.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L = 4096
    n = 10_000_000
    d = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    s = torch.cuda.current_stream()
    sp = ctypes.c_void_p(s.cuda_stream)
    assert lb.lsbm_fill_splitmix64_dev(ctypes.c_void_p(d.data_ptr()), n * L, 0x5EED0000, sp) == 0
    out = torch.empty(n, dtype=torch.int32, device="cuda")
    st = np.zeros((4, 65536), dtype=np.uint64)
    for m in (1 << 20, n, 1 << 20, n):
        def launch():
            assert lb.lsbm_crc32c_fixed_dev(ctypes.c_void_p(d.data_ptr()), L, L, m, None,
                                            ctypes.c_void_p(out.data_ptr()), 0, sp) == 0
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < 0.3:
            launch()
            torch.cuda.synchronize()
        launch()
        torch.cuda.synchronize()
        assert lb.lsbm_diag_stamps(st.ctypes.data, 4 * 65536) == 0
        cus = torch.cuda.get_device_properties(0).multi_processor_count
        nw = int(np.count_nonzero(st[2]))
        nw = min(nw, 65536)
        start, end = st[0][:nw].astype(np.int64), st[2][:nw].astype(np.int64)
        t0 = start.min()
        dur = (end - start) / 100.0  # us
        endr = (end - t0) / 100.0
        span = endr.max()
        rec = {"blocks": m, "waves": nw, "cus": cus, "span_us": round(float(span), 1),
               "GBps_span": round(m * L / (span / 1e6) / 1e9, 1),
               "start_spread_us": round(float((start - t0).max() / 100.0), 1),
               "end_p0_p10_p50_p90_p100_us": [round(float(x), 1) for x in np.percentile(endr, [0, 10, 50, 90, 100])],
               "dur_mean_us": round(float(dur.mean()), 1),
               "dur_cv": round(float(dur.std() / dur.mean()), 4),
               "dur_min_max_us": [round(float(dur.min()), 1), round(float(dur.max()), 1)],
               # time the GPU is not fully busy: after the first wave ends
               "tail_us": round(float(span - endr.min()), 1),
               "tail_frac": round(float((span - endr.min()) / span), 4),
               # how far apart the fastest and the slowest wave are at the end (bytes of the batch)
               "window_spread_MiB": round(float((dur.max() - dur.min()) / dur.max() * m * L / 2**20), 1)}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
