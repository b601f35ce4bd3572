"""Diagnostic: group [325, 350) of the failing case alone, and prefixes of it."""
import os, sys
import numpy as np
REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO); sys.path.insert(0, os.path.join(REPO, "tests"))
import torch
from conftest import BloomOracle
from golden.bloomkeys import take, random_keys
from test_bloom import gpu_build
o = BloomOracle(os.path.join(REPO, "oracle", "liboracle_bloom.so"))
bits_per_key, strip, gap = 10, 8, 3
rng = np.random.default_rng(bits_per_key * 7 + strip)
counts = rng.integers(0, 80, size=400)
counts[::50] = rng.integers(300, 3000, size=counts[::50].size)
counts[5] = 0
n = int(counts.sum())
keys = random_keys(1000 + bits_per_key, n, strip, strip + 40)
first = np.concatenate([[0], np.cumsum(counts)])

def run(fids, label):
    filters = [(int(first[i]), int(first[i + 1])) for i in fids]
    out, offs, sizes = gpu_build(torch, keys, filters, bits_per_key, strip, gap)
    bad = []
    for j, (k0, k1) in enumerate(filters):
        want = o.create_filter(take(keys, range(k0, k1)), bits_per_key, strip)
        got = out[int(offs[j]):int(offs[j]) + sizes[j]].tobytes()
        if got != want:
            bad.append(fids[j])
    print(label, len(fids), "bad", bad, flush=True)

run(list(range(325, 350)), "group")
for m in (1, 2, 5, 10, 17, 24):
    run(list(range(325, 325 + m)), f"prefix{m}")
run(list(range(326, 350)), "from326")
run(list(range(275, 300)), "group275")
