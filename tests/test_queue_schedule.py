"""The fixed kernel's cross-XCC work-queue schedule (crc32c_kernels.hip,
crc32c_units.h queue_issue / queue_resolve), restated step for step on the
CPU: waves run in random order; each wave's first group is its own (row 0 of
the interleave); past it, items of k groups are claimed from 8 per-XCC heads
(head h hands out items 8 j + h), one claim issued in the last group of the
current item (behind its last row loads; the item may end early at the batch
end) and resolved after it, and a wave whose head is exhausted
moves on to the next head.  Every group must be processed exactly once,
every resolve must consume the claim issued for its own item (no stale
claim: round 6's first multi-group version re-resolved one and looped), and
every wave must stop."""
import random

import pytest


def simulate(ngroups, nwaves, k, seed):
    rnd = random.Random(seed)
    heads = [0] * 8
    q_items = (ngroups - nwaves + k - 1) // k if ngroups > nwaves else 0
    waves = [dict(grp=w, qh=rnd.randrange(8), pend=None, out=0, q_end=w + 1, steps=0)
             for w in range(nwaves)]
    seen = [0] * ngroups

    def issue(h):
        j = heads[h]
        heads[h] += 1
        return j

    def resolve(wv):
        assert wv["pend"] is not None, "resolve without a claim of its own"
        item = wv["pend"] * 8 + wv["qh"]
        wv["pend"] = None
        while item >= q_items:
            wv["out"] += 1
            if wv["out"] >= 8:
                return q_items
            wv["qh"] = (wv["qh"] + 1) % 8
            item = issue(wv["qh"]) * 8 + wv["qh"]
        return item

    active = [w for w in waves if w["grp"] < ngroups]
    while active:
        wv = rnd.choice(active)
        wv["steps"] += 1
        assert wv["steps"] < 10 * ngroups + 100, "no progress"
        g = wv["grp"]
        if g + 1 == wv["q_end"] or g + 1 == ngroups:  # q_last: the item's last group
            assert wv["pend"] is None, "two claims for one item"
            wv["pend"] = issue(wv["qh"])
        seen[g] += 1
        wv["grp"] += 1
        if wv["grp"] >= wv["q_end"] or wv["grp"] >= ngroups:
            it = resolve(wv)
            wv["grp"] = nwaves + it * k if it < q_items else ngroups
            wv["q_end"] = wv["grp"] + k
        if wv["grp"] >= ngroups:
            active.remove(wv)
    return seen


@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_every_group_once(k):
    for seed in range(80):
        r = random.Random(seed * 7 + k)
        nw = r.choice([1, 3, 16, 64, 200])
        ng = r.choice([0, 1, nw, nw + 1, nw * 4 + 3, r.randrange(1, 3000)])
        seen = simulate(ng, nw, k, seed)
        assert all(s == 1 for s in seen), (ng, nw, k, seed)
