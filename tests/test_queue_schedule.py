"""The fixed kernel's cross-XCC work queue (crc32c_units.h WgQueue, used by
crc32c_fixed_kernel), restated step for step on the CPU and run under random
interleavings of the waves.

Each workgroup's W waves first take their own group of row 0; then they take
slots k = W, W+1, ... from an LDS counter: slot k is wave-group k % W of batch
k / W.  Batch b's item is claimed from 8 per-XCC heads (head h hands out items
8 j + h; an exhausted head sends the workgroup on to the next one) by the wave
that took slot 0 of batch b - kLead, and published through a ring of kRing
LDS entries: publish(x) waits until batch x - 1 is published (claims in batch
order) and until all W readers of batch x - kRing have read the entry it
reuses; a reader spins until its batch's tag appears, counts itself as read,
and stops at the first exhausted batch (kNone).  Checked: every group is
processed exactly once, no entry is overwritten before all its readers read it,
and every wave stops (no wait cycle).  Round 6's first version (publication in
any order) lost items claimed after an exhausted one; so did reading a batch-0
entry nobody publishes -- this test found both before any GPU run."""
import random

import pytest

NONE = -1


def simulate(ngroups, nwg, W, lead, ring, seed):
    rnd = random.Random(seed)
    nwaves = nwg * W
    items = (ngroups - nwaves + W - 1) // W if ngroups > nwaves else 0
    heads = [0] * 8
    seen = [0] * ngroups
    wgs = [dict(next=W, h=rnd.randrange(8), out=0, tag=[0] * ring, item=[NONE] * ring, read=[0] * ring)
           for _ in range(nwg)]

    def claim(S):  # WgQueue::publish's head loop
        while S["out"] < 8:
            j = heads[S["h"]]
            heads[S["h"]] += 1
            it = j * 8 + S["h"]
            if it < items:
                return it
            S["out"] += 1
            if S["out"] < 8:
                S["h"] = (S["h"] + 1) % 8
        return NONE

    waves = [dict(wg=b, st="own", k=None, pub=lead if w == 0 else 0, done=False)
             for b in range(nwg) for w in range(W)]
    for wv in waves:
        wv["grp"] = wv["wg"] * W + waves.index(wv) % W  # row 0: the wave's own group
    active = list(waves)
    steps = 0
    while active:
        steps += 1
        assert steps < 200 * (ngroups + nwaves) + 10000, "a wait cycle"
        wv = rnd.choice(active)
        S = wgs[wv["wg"]]
        if wv["st"] == "own":  # row 0 (its loads were issued before the tables)
            if wv["pub"]:
                wv["st"] = "publish_then_work"
            else:
                wv["st"] = "work"
        if wv["st"] in ("publish_then_work", "publish_then_exit"):
            x = wv["pub"]
            e, pe = x % ring, (x - 1) % ring
            if x >= 2 and S["tag"][pe] != x - 1:
                continue  # spin: batch order
            if x > ring and S["read"][e] != W:
                continue  # spin: the entry's previous batch not read by all yet
            assert x <= ring or S["tag"][e] == x - ring
            it = claim(S)
            S["item"][e], S["read"][e], S["tag"][e] = it, 0, x
            wv["pub"] = 0
            if wv["st"] == "publish_then_exit":
                wv["done"] = True
                active.remove(wv)
                continue
            wv["st"] = "work"
            continue
        if wv["st"] == "work":
            if wv["grp"] < ngroups:
                seen[wv["grp"]] += 1
            k = S["next"]
            S["next"] += 1
            wv["k"] = k
            if k % W == 0:
                wv["pub"] = k // W + lead
            wv["st"] = "read"
            continue
        if wv["st"] == "read":
            b, slot = wv["k"] // W, wv["k"] % W
            e = b % ring
            if S["tag"][e] != b:
                assert S["tag"][e] < b, "entry overwritten before it was read"
                continue  # spin
            it = S["item"][e]
            S["read"][e] += 1
            if it == NONE:
                if wv["pub"]:
                    wv["st"] = "publish_then_exit"
                else:
                    active.remove(wv)
                continue
            wv["grp"] = nwaves + it * W + slot
            wv["st"] = "publish_then_work" if wv["pub"] else "work"
    return seen


@pytest.mark.parametrize("lead,ring", [(1, 4), (1, 2), (1, 3), (1, 8)])
def test_every_group_once(lead, ring):
    for seed in range(150):
        r = random.Random(seed * 31 + lead * 7 + ring)
        W = r.choice([1, 2, 4, 16])
        nwg = r.choice([1, 2, 8, 24])
        nw = nwg * W
        ng = r.choice([0, 1, nw, nw + 1, nw + W * 8 * 3 + 5, r.randrange(1, 4000)])
        seen = simulate(ng, nwg, W, lead, ring, seed)
        assert all(s == 1 for s in seen), (ng, nwg, W, lead, ring, seed)


def test_kernel_constants_match():
    """The simulated lead and ring include the kernel's (crc32c_units.h)."""
    import os
    import re
    src = open(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                            "lsbm_amd", "csrc", "crc32c_units.h")).read()
    m = re.search(r"kWqRing = (\d+), kWqLead = (\d+)", src)
    assert m and (int(m.group(2)), int(m.group(1))) == (1, 4)
