#!/usr/bin/env python3
"""Timing/traffic-only ablations of the inflate wave kernel (VERDICT r5 item
1b): each variant is the product source with one class of global accesses
removed, built into variants/<name>.so.  The output of an ablated build is
wrong by construction; they exist only to split the kernel's fabric traffic
(tools/iw_traffic_split.sh) and time by phase.  Product sources are never
edited.
  nofar   far-token source pieces are not loaded (the stores stay)
  nonsrc  near bytes whose source lies before the stage do not load it
  nofs    both
"""
import os, subprocess, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
C = os.path.join(R, "zarr_amd", "csrc")
SRC = open(os.path.join(C, "zcg_inflate_wave.hip")).read()
FAR = [("V0 = *(const gu32x4_ua*)(gd + src);", "V0 = u32x4{src, src ^ 1u, src ^ 2u, src ^ 3u};"),
       ("V1 = *(const gu32x4_ua*)(gd + src + (np > 1 ? 16u : 0u));", "V1 = V0;"),
       ("const u32x4 Vp = *(const gu32x4_ua*)(gd + src + 16 * p);", "const u32x4 Vp = V0 + p;")]
NSRC = [("else cur = IE_VAL | (u32)gd[swap_pos32(S32 + p - d, tw)];", "else cur = IE_VAL | (p & 0xFFu);")]  # (!wide_ok only since round 6)
VARIANTS = {"nofar": FAR, "nonsrc": NSRC, "nofs": FAR + NSRC}


def main(names):
    os.makedirs(os.path.join(R, "variants"), exist_ok=True)
    subprocess.run(["make", "-s", "-j8", "-C", C], check=True)
    objs = sorted(os.path.join(C, "build", f) for f in os.listdir(os.path.join(C, "build"))
                  if f.endswith(".o") and f != "zcg_inflate_wave.o")
    for name in names:
        s = SRC
        for a, b in VARIANTS[name]:
            assert s.count(a) == 1, (name, a)
            s = s.replace(a, b)
        d = os.path.join(R, "variants", "obj_" + name)
        os.makedirs(d, exist_ok=True)
        sp = os.path.join(d, "zcg_inflate_wave.hip")
        open(sp, "w").write(s)
        o = os.path.join(d, "zcg_inflate_wave.o")
        subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-fPIC", "-std=c++17", "--offload-arch=gfx950",
                        "-munsafe-fp-atomics", "-I" + C, "-I" + os.path.join(R, "include"), "-c", sp, "-o", o],
                       check=True)
        subprocess.run(["/opt/rocm/bin/hipcc", "-shared", "-fPIC", "--offload-arch=gfx950", "-o",
                        os.path.join(R, "variants", name + ".so")] + objs + [o], check=True)
        print("built variants/%s.so" % name)


if __name__ == "__main__":
    main(sys.argv[1:] or list(VARIANTS))
