"""Per-tile phase timeline of the single-pass IIR kernel (development tool). Needs the timing build:
    tools/variant_lib.sh timing gsdr_amd/csrc/iir.hip -DGSDR_TUNING_PROBES -DGSDR_IIR_RES_TIMING
which writes each tile's wall-clock marks (100 MHz) over the first words of its output instead of y.
Prints per-phase medians for 2^24 samples (4th / 8th-order Butterworth, real and complex)."""
import ctypes, os, sys, numpy as np, torch
from scipy import signal as sps
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "build", "var_timing", "libgsdr.so"))
dev = torch.device("cuda:0")
n = 1 << 24
P = ctypes.c_void_p
out = {}
for name, K, order, cplx in (("FF5", 5, 4, False), ("CC5", 5, 4, True), ("FF9", 9, 8, False)):
    bb, aa = (torch.tensor(v, dtype=torch.float32, device=dev) for v in sps.butter(order, 0.1))
    x = torch.rand(2 * n if cplx else n, device=dev)
    y = torch.empty_like(x)
    st = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    fn = lib.gsdrxIirCCSinglePass if cplx else lib.gsdrxIirFFSinglePass
    for _ in range(5):
        fn(P(bb.data_ptr()), P(aa.data_ptr()), ctypes.c_size_t(K), None, None, P(x.data_ptr()), P(y.data_ptr()), ctypes.c_size_t(n),
           ctypes.c_uint32(1 << 22), 0, st)
    torch.cuda.synchronize()
    TS = 4096 if cplx else 8192   # samples a tile
    per = TS * (2 if cplx else 1)  # floats a tile
    yv = y.cpu().numpy().view(np.uint32)
    nt = n // TS
    ts = np.stack([yv[t * per: t * per + 26].view(np.uint64) for t in range(nt)])  # [tile][13]
    t0 = ts[:, 0].min()
    rel = (ts[:, :9] - t0) / 100.0  # 100 MHz -> us
    d = np.diff(rel, axis=1)
    print(name, "tiles", nt, "kernel span us %.1f" % rel[:, 8].max())
    print("  phase medians us (M0, sq+stage, pass1, scan+publish, wait, U/Q/compose, fix, store):", np.round(np.median(d, 0), 2))
    print("  phase p90:", np.round(np.percentile(d, 90, 0), 2))
    print("  start quantiles:", np.round(np.percentile(rel[:, 0], [0, 10, 25, 50, 75, 90, 100]), 1))
    nl = np.array([(k % 256) != 255 for k in range(nt)])
    sub = (ts[nl][:, [5, 9, 10, 11]].astype(np.int64) - ts[nl][:, [5]].astype(np.int64)) / 100.0
    print("  non-last compose split (poll done, mat_pows done, sum done) after ts5, medians:", np.round(np.median(sub, 0), 2), "p90", np.round(np.percentile(sub, 90, 0), 2))
    print("  tile duration median %.1f p90 %.1f" % (np.median(rel[:, 8] - rel[:, 0]), np.percentile(rel[:, 8] - rel[:, 0], 90)))
    np.save("gpurun_out/iir_ts_%s.npy" % name, ts)
