import random
def sim(ngroups, nwaves, k, seed):
    rnd = random.Random(seed)
    heads = [0]*8
    q_items = (ngroups - nwaves + k - 1)//k if ngroups > nwaves else 0
    waves = []
    for w in range(nwaves):
        waves.append(dict(grp=w, qh=rnd.randrange(8), pend=None, out=0, q_start=w, q_end=w+1, done=False, steps=0))
    seen = [0]*ngroups
    def issue(h):
        j = heads[h]; heads[h] += 1; return j
    def resolve(wv):
        item = wv['pend']*8 + wv['qh']
        assert wv['pend'] is not None
        wv['pend'] = None
        while item >= q_items:
            wv['out'] += 1
            if wv['out'] >= 8: return q_items
            wv['qh'] = (wv['qh']+1) % 8
            item = issue(wv['qh'])*8 + wv['qh']
        return item
    active = [w for w in waves if w['grp'] < ngroups]
    while active:
        wv = rnd.choice(active)
        wv['steps'] += 1
        assert wv['steps'] < 10*ngroups+100, "no progress"
        g = wv['grp']
        if g == wv['q_start']:
            assert wv['pend'] is None
            wv['pend'] = issue(wv['qh'])
        seen[g] += 1
        wv['grp'] += 1
        if wv['grp'] >= wv['q_end'] or wv['grp'] >= ngroups:
            it = resolve(wv)
            wv['grp'] = nwaves + it*k if it < q_items else ngroups
            wv['q_start'] = wv['grp']; wv['q_end'] = wv['grp'] + k
        if wv['grp'] >= ngroups: active.remove(wv)
    assert all(s == 1 for s in seen), (ngroups, nwaves, k, [i for i,s in enumerate(seen) if s != 1][:5])
for seed in range(300):
    r = random.Random(seed)
    nw = r.choice([1, 3, 16, 64, 200])
    ng = r.choice([0, 1, nw, nw+1, nw*4+3, r.randrange(1, 3000)])
    k = r.choice([1, 2, 3, 4])
    sim(ng, nw, k, seed)
print("ok")
