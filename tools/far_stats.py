#!/usr/bin/env python3
"""Token-level model of one C2 chunk for the inflate wave kernel's L phase
(CPU only, pure-Python deflate parser tools/deflate_tokens.py): literal / far
/ near token counts and lengths with stages of <= 2032 bytes ending at token
boundaries, the far-distance distribution, and the distinct 128-byte source
lines the far parts of each stage touch.  usage: far_stats.py [chunk index]"""
import collections
import os
import sys
import zlib

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, HERE)
from bench import quant_chunk  # noqa: E402
import deflate_tokens as dt  # noqa: E402

CAP = 2032
v = quant_chunk(int(sys.argv[1]) if len(sys.argv) > 1 else 0).tobytes()
toks = dt.tokens(zlib.compress(v, 6)[2:-4])
lit = far = near = farb = nearb = 0
fard, lines_per_stage, cur = [], [], set()
pos = S = 0
for t in toks:
    L = 1 if t[0] == 'L' else t[1]
    if pos + L - S > CAP:
        lines_per_stage.append(len(cur))
        cur, S = set(), pos
    if t[0] == 'L':
        lit += 1
    else:
        d, o = t[2], pos - S
        if o + L <= d:
            far += 1
            farb += L
            fard.append(d)
            a = pos - d
            for ln in range(a // 128, (a + max(L, 16) - 1) // 128 + 1):
                cur.add(ln)
        else:
            near += 1
            nearb += L
    pos += L
fard = np.array(fard)
print({"tokens": len(toks), "literals": lit, "far_tokens": far, "far_bytes": farb, "near_tokens": near,
       "near_bytes": nearb, "stages": len(lines_per_stage),
       "far_distance_le": {q: round(float((fard <= q).mean()), 3) for q in (2048, 4096, 8192, 16384, 32768)},
       "far_lines_per_stage": round(float(np.mean(lines_per_stage)), 1),
       "far_line_bytes_per_chunk": int(sum(lines_per_stage) * 128)})
