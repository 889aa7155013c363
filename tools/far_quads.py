#!/usr/bin/env python3
"""Token-level model of the inflate wave kernel's far-byte gather on one C2
chunk: a pure-Python deflate token parser, stages of <= 2048 bytes ending at
token boundaries, and per 4-entry quad of a lane block the loads the gather
needs (consecutive-quad rule vs a 4-byte-span rule).  CPU only.
  usage: far_quads.py [chunk index]"""
import sys, zlib, numpy as np
sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from bench import quant_chunk
class BR:
    def __init__(s, b): s.b = b; s.p = 0
    def bits(s, n):
        v = 0
        for i in range(n):
            v |= ((s.b[s.p >> 3] >> (s.p & 7)) & 1) << i; s.p += 1
        return v
def mk(lens):
    codes = {}; code = 0; bl = [0]*16
    for l in lens:
        if l: bl[l] += 1
    nxt = [0]*16
    for b in range(1, 16):
        code = (code + bl[b-1]) << 1; nxt[b] = code
    for i, l in enumerate(lens):
        if l: codes[(l, nxt[l])] = i; nxt[l] += 1
    return codes
def dec(br, t):
    c = 0; l = 0
    while True:
        c = (c << 1) | br.bits(1); l += 1
        if (l, c) in t: return t[(l, c)]
LB = [3,4,5,6,7,8,9,10,11,13,15,17,19,23,27,31,35,43,51,59,67,83,99,115,131,163,195,227,258]
LE = [0,0,0,0,0,0,0,0,1,1,1,1,2,2,2,2,3,3,3,3,4,4,4,4,5,5,5,5,0]
DB = [1,2,3,4,5,7,9,13,17,25,33,49,65,97,129,193,257,385,513,769,1025,1537,2049,3073,4097,6145,8193,12289,16385,24577]
DE = [0,0,0,0,1,1,2,2,3,3,4,4,5,5,6,6,7,7,8,8,9,9,10,10,11,11,12,12,13,13]
def tokens(raw):
    br = BR(raw); out = []
    while True:
        last = br.bits(1); ty = br.bits(2)
        if ty == 0:
            br.p = (br.p + 7) & ~7; n = br.bits(16); br.bits(16)
            out += [('L', 0)] * n; br.p += 8 * n
        else:
            if ty == 1:
                lt = mk([8]*144 + [9]*112 + [7]*24 + [8]*8); dt = mk([5]*30)
            else:
                hl = br.bits(5) + 257; hd = br.bits(5) + 1; hc = br.bits(4) + 4
                order = [16,17,18,0,8,7,9,6,10,5,11,4,12,3,13,2,14,1,15]
                cl = [0]*19
                for i in range(hc): cl[order[i]] = br.bits(3)
                ct = mk(cl); ls = []
                while len(ls) < hl + hd:
                    s = dec(br, ct)
                    if s < 16: ls.append(s)
                    elif s == 16: ls += [ls[-1]] * (3 + br.bits(2))
                    elif s == 17: ls += [0] * (3 + br.bits(3))
                    else: ls += [0] * (11 + br.bits(7))
                lt = mk(ls[:hl]); dt = mk(ls[hl:])
            while True:
                s = dec(br, lt)
                if s < 256: out.append(('L', 0))
                elif s == 256: break
                else:
                    s -= 257; ln = LB[s] + br.bits(LE[s])
                    ds = dec(br, dt); d = DB[ds] + br.bits(DE[ds])
                    out.append(('M', ln, d))
        if last: return out
v = quant_chunk(int(sys.argv[1]) if len(sys.argv) > 1 else 0).tobytes()
c = zlib.compressobj(6, zlib.DEFLATED, -15); raw = c.compress(v) + c.flush()
tk = tokens(raw)
# per output byte: (token start, dist) or literal
N = len(v); mo = np.zeros(N, np.int64); md = np.zeros(N, np.int64); x = 0
starts = []
for t in tk:
    starts.append(x)
    if t[0] == 'L': md[x] = 0; x += 1
    else:
        mo[x:x+t[1]] = x; md[x:x+t[1]] = t[2]; x += t[1]
starts.append(x)
assert x == N, (x, N)
import bisect
S = 0; cur = 0; nq = 0; q_old = 0; q_new = 0; q_new8 = 0; far_e = 0
while S < N:
    cap = 2048 - (S & 31); lim = S + cap
    j = bisect.bisect_right(starts, lim) - 1
    E = max(starts[j], S + 1) if starts[j] > S else min(N, lim)
    if E <= S: E = min(N, S + cap)
    B0 = S & ~31
    for blk in range(B0, E, 32):
        for q0 in range(blk, blk + 32, 4):
            src = []
            for xx in range(q0, q0 + 4):
                if xx < S or xx >= E or md[xx] == 0: src.append(None); continue
                d = md[xx]; m = mo[xx]; sp = m - d + ((xx - m) % d)
                src.append(sp if sp < S else None)
            fs = [s for s in src if s is not None]
            if not fs: continue
            nq += 1; far_e += len(fs)
            cons = len(fs) == 4 and all(src[k] == src[0] + k for k in range(4))
            q_old += 1 if cons else len(fs)
            q_new += 1 if max(fs) - min(fs) < 4 else len(fs)
    S = E
print(dict(tokens=len(tk), far_entries=far_e, far_quads=nq, loads_now=q_old, loads_span4=q_new))
