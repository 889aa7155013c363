"""Pure-Python deflate token parser (raw deflate -> [('L',0) | ('M', len, dist)]).
Model/statistics tooling only (CPU); not used by the product or the tests."""
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
