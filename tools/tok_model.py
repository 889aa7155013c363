#!/usr/bin/env python3
"""Token-level model of the inflate wave kernel's L phase on one C2 chunk:
stages of <= 2048 bytes ending at token boundaries (the kernel's cut rule),
and per stage the literal / far-match / near-match token counts, the near
bytes, and the token-level dependency depth of the near matches (a near match
whose source touches an unresolved near match is one level deeper).  Used to
price a token-granular far copy against today's per-byte entries.  CPU only.
  usage: tok_model.py [chunk index]"""
import bisect
import os
import sys
import zlib

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import quant_chunk  # noqa: E402
from deflate_tokens import tokens  # noqa: E402

v = quant_chunk(int(sys.argv[1]) if len(sys.argv) > 1 else 0).tobytes()
c = zlib.compressobj(6, zlib.DEFLATED, -15)
raw = c.compress(v) + c.flush()
tk = tokens(raw)
starts = []
x = 0
for t in tk:
    starts.append(x)
    x += 1 if t[0] == 'L' else t[1]
N = x
starts.append(N)
st = dict(stages=0, lit=0, far=0, far_ovl=0, near=0, near_bytes=0, far_bytes=0, far_dwords=0, far_dwords_ovl=0)
depth_hist = {}
len_hist = {}
dist_small = 0
near_src_in_near = 0
ti = 0
S = 0
maxdepth_per_stage = []
while S < N:
    cap = 2048 - (S & 31)
    lim = S + cap
    j = bisect.bisect_right(starts, lim) - 1
    E = starts[j] if starts[j] > S else min(N, lim)
    st['stages'] += 1
    # tokens in [S, E)
    lvl = {}  # output byte -> depth of the near token writing it (0 = resolved by literal/far)
    md = 0
    while ti < len(tk) and starts[ti] < E:
        o = starts[ti]
        t = tk[ti]
        if t[0] == 'L':
            st['lit'] += 1
        else:
            L, d = t[1], t[2]
            len_hist[L] = len_hist.get(L, 0) + 1
            if d < 4:
                dist_small += 1
            a = o - d
            span = min(L, d)
            if a + span <= S:
                st['far'] += 1
                st['far_bytes'] += L
                st['far_dwords'] += ((o + L + 3) // 4) - (o // 4)
                if d < L:
                    st['far_ovl'] += 1
            else:
                st['near'] += 1
                st['near_bytes'] += L
                dep = 1
                for y in range(max(a, S), a + span):
                    dep = max(dep, lvl.get(y, 0) + 1)
                if dep > 1:
                    near_src_in_near += 1
                for y in range(o, o + L):
                    lvl[y] = dep
                depth_hist[dep] = depth_hist.get(dep, 0) + 1
                md = max(md, dep)
        ti += 1
    maxdepth_per_stage.append(md)
    S = E
print(dict(tokens=len(tk), **st, dist_lt4=dist_small, near_src_in_near=near_src_in_near))
print('near depth hist', sorted(depth_hist.items()))
h = np.bincount(np.array(maxdepth_per_stage))
print('max near depth per stage hist', list(enumerate(h.tolist())))
print('len hist (top)', sorted(len_hist.items(), key=lambda kv: -kv[1])[:16])

# ---- cost model of a token-granular L phase (groups of 128 tokens, lane l
# holds tokens 2l and 2l + 1 of a group; a group never crosses a stage) ----
S = 0
ti = 0
far_it = 0; near_it = 0; groups = 0; nbatches = 0; fq_tot = 0; nb_tot = 0; stages = 0
far_it_split = 0
while S < N:
    cap = 2048 - (S & 31)
    lim = S + cap
    j = bisect.bisect_right(starts, lim) - 1
    E = starts[j] if starts[j] > S else min(N, lim)
    stages += 1
    stoks = []
    while ti < len(tk) and starts[ti] < E:
        stoks.append((starts[ti], tk[ti])); ti += 1
    nb = 0
    for g0 in range(0, len(stoks), 128):
        grp = stoks[g0:g0 + 128]
        groups += 1
        fq = [0] * 64; nbk = [0] * 64
        for i, (o, t) in enumerate(grp):
            if t[0] == 'L':
                continue
            L, d = t[1], t[2]
            if o - d + min(L, d) <= S and d >= L:
                q = (o + L + 3) // 4 - o // 4
                fq[i // 2] += q; fq_tot += q
            else:
                nbk[i // 2] += L; nb += L
        far_it += max(fq); near_it += max(nbk)
        far_it_split += -(-sum(fq) // 64)
    nb_tot += nb
    nbatches += -(-nb // 64)
    S = E
print(dict(stages=stages, groups=groups, far_iter_per_stage=far_it / stages, far_iter_balanced=far_it_split / stages,
           far_quads_per_stage=fq_tot / stages, near_iter_per_stage=near_it / stages,
           near_bytes_per_stage=nb_tot / stages, near_batches_per_stage=nbatches / stages))

# ---- near tokens whose source lies before their group's first byte (settled) ----
S = 0; ti = 0; settled = 0; nearc = 0; settled_b = 0; near_b = 0; st16 = 0
while S < N:
    cap = 2048
    lim = S + cap
    j = bisect.bisect_right(starts, lim) - 1
    E = starts[j] if starts[j] > S else min(N, lim)
    stoks = []
    while ti < len(tk) and starts[ti] < E:
        stoks.append((starts[ti], tk[ti])); ti += 1
    for g0 in range(0, len(stoks), 128):
        grp = stoks[g0:g0 + 128]
        og = grp[0][0]
        for (o, t) in grp:
            if t[0] == 'L':
                continue
            L, d = t[1], t[2]
            if o - d + min(L, d) <= S and d >= L:
                continue
            nearc += 1; near_b += L
            if o - d + min(L, d) <= og and o - d >= S:
                settled += 1; settled_b += L
                if L <= 16: st16 += 1
    S = E
print(dict(near=nearc, settled=settled, near_bytes=near_b, settled_bytes=settled_b, settled_le16=st16))
