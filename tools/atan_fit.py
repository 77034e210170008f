# Development tool: fit of the odd polynomial used by disc_atan2 (gsdr_amd/csrc/fir_engine.hpp) and its
# max abs error when evaluated in float32 (Lawson-weighted least squares toward minimax).
import numpy as np
# fit atan(t)/t = P(s), s = t^2, t in [0,1], weighted least squares on Chebyshev nodes, then check float32 eval
for deg in (4, 5, 6, 7):
    t = np.cos(np.pi * (np.arange(4000) + 0.5) / 4000) * 0.5 + 0.5
    s = t * t
    f = np.arctan(t) / np.where(t == 0, 1, t)
    f[t == 0] = 1
    # minimize absolute error of t*P(s): weight rows by t
    A = np.stack([s ** k for k in range(deg)], 1) * t[:, None]
    c, *_ = np.linalg.lstsq(A, np.arctan(t), rcond=None)
    # a few Lawson iterations toward minimax
    w = np.ones_like(t)
    for it in range(50):
        c, *_ = np.linalg.lstsq(A * w[:, None], np.arctan(t) * w, rcond=None)
        e = np.abs(A @ c - np.arctan(t))
        w = w * (e / e.max() + 1e-3) ** 0.5
        w /= w.mean()
    c32 = c.astype(np.float32)
    tt = np.linspace(0, 1, 2000001).astype(np.float32)
    ss = (tt * tt).astype(np.float32)
    p = np.float32(c32[-1])
    for k in range(deg - 2, -1, -1):
        p = (p * ss + c32[k]).astype(np.float32)
    r = (p * tt).astype(np.float32)
    err = np.max(np.abs(r.astype(np.float64) - np.arctan(tt.astype(np.float64))))
    print(deg, err, [float(v) for v in c32])
