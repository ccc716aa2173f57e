"""Round 5 diagnostic: tools/r05/trig_probe's device results against the host C library
(glibc atan2f / sinf / cosf through ctypes, which the reference's 1-element torch ops
call). Usage: trig_compare.py trig_in.bin trig_out.bin"""
import ctypes
import sys

import numpy as np

libm = ctypes.CDLL("libm.so.6")
for fn in ("sinf", "cosf"):
    getattr(libm, fn).argtypes = [ctypes.c_float]
    getattr(libm, fn).restype = ctypes.c_float
libm.atan2f.argtypes = [ctypes.c_float, ctypes.c_float]
libm.atan2f.restype = ctypes.c_float


def main(fin, fout, nsample=200_000):
    with open(fin, "rb") as f:
        na, nt = np.fromfile(f, np.int32, 2)
        yx = np.fromfile(f, np.float32, 2 * na).reshape(na, 2)
        th = np.fromfile(f, np.float32, nt)
    out = np.fromfile(fout, np.float32)
    at = out[:na]
    tr = out[na:].reshape(nt, 4)
    h_at = np.array([libm.atan2f(float(a), float(b)) for a, b in yx], np.float32)
    print(f"atan2f (segment normal angles, {na}): device != glibc on {np.sum(at != h_at)}")
    idx = np.random.default_rng(0).choice(nt, min(nsample, nt), replace=False)
    hs = np.array([libm.sinf(float(t)) for t in th[idx]], np.float32)
    hc = np.array([libm.cosf(float(t)) for t in th[idx]], np.float32)
    for j, name in enumerate(("sinf (OCML)", "cosf (OCML)", "__sinf (v_sin)", "__cosf (v_cos)")):
        ref = hs if j % 2 == 0 else hc
        d = tr[idx, j]
        ne = d != ref
        ulp = np.abs(d.astype(np.float64) - ref) / np.spacing(np.maximum(np.abs(ref), np.float32(1e-30)))
        print(f"{name:15s}: != glibc on {ne.mean():.5f} of {len(idx)} angles, max {ulp.max():.1f} ulp"
              f" (of |ref|), p99 {np.quantile(ulp, 0.99):.2f}")


if __name__ == "__main__":
    main(*sys.argv[1:3])
