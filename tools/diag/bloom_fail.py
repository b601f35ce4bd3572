"""Diagnostic: the failing test_gpu_build_matches_oracle[8-3-10] case; prints
every filter that differs from the oracle and how."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch
from conftest import BloomOracle
from golden.bloomkeys import take
from golden.bloomkeys import random_keys
from test_bloom import gpu_build
o = BloomOracle(os.path.join(REPO, "oracle", "liboracle_bloom.so"))
for bits_per_key, strip, gap in [(10, 8, 3), (10, 0, 0), (20, 8, 3), (3, 8, 3)]:
    rng = np.random.default_rng(bits_per_key * 7 + strip)
    counts = rng.integers(0, 80, size=400)
    counts[::50] = rng.integers(300, 3000, size=counts[::50].size)
    counts[5] = 0
    n = int(counts.sum())
    keys = random_keys(1000 + bits_per_key, n, strip, strip + 40)
    filters, k = [], 0
    for c in counts:
        filters.append((k, k + int(c)))
        k += int(c)
    out, offs, sizes = gpu_build(torch, keys, filters, bits_per_key, strip, gap)
    bad = []
    for i, (k0, k1) in enumerate(filters):
        want = o.create_filter(take(keys, range(k0, k1)), bits_per_key, strip)
        got = out[int(offs[i]):int(offs[i]) + sizes[i]].tobytes()
        if got != want:
            nb = sum(bin(a ^ b).count("1") for a, b in zip(got, want))
            bad.append((i, int(counts[i]), sizes[i], nb))
    print(bits_per_key, strip, gap, "bad:", bad[:20], len(bad), flush=True)
