"""Stand-alone timing of the fused V-trace kernel through the C ABI (no learner around it).

usage: python scripts/vtrace_bench.py [--lib path/to/libfi_learner.so ...] [--T 100 --B 4096 --A 18]
Prints one line per library: mean launch time (HIP events over --iters back-to-back launches,
finalize included) and the algorithmic HBM rate (12A+28 bytes per (t,b)).
Several --lib values let experiment builds be compared in one GPU session.
"""
import argparse
import ctypes as C
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", default=[])
    ap.add_argument("--T", type=int, default=100)
    ap.add_argument("--B", type=int, default=4096)
    ap.add_argument("--A", type=int, default=18)
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--variant", type=int, action="append", default=[],
                    help="kernel variant(s) to time (0 auto, 1 chunked LDS, 2 column, 3 whole-sequence)")
    ap.add_argument("--sets", type=int, default=1, help="rotate over this many disjoint input/output sets (6: cold)")
    ap.add_argument("--stamps", action="store_true",
                    help="libs built with -DFI_VT_STAMPS: print per-phase timing of wave 0")
    args = ap.parse_args()
    from freeimpala_amd import _abi, hip
    libs = args.lib or [None]
    T, B, A = args.T, args.B, args.A
    rng = np.random.default_rng(0)
    pi = rng.standard_normal((T, B, A), dtype=np.float32)
    mu = rng.standard_normal((T, B, A), dtype=np.float32)
    act = rng.integers(0, A, (T, B), dtype=np.int32)
    rew = rng.integers(-1, 2, (T, B)).astype(np.float32)
    disc = (0.99 * (rng.random((T, B)) > 0.01)).astype(np.float32)
    val = rng.standard_normal((T + 1, B), dtype=np.float32)
    nsets = max(1, args.sets)
    bufs = [[hip.DeviceBuffer.from_array(x) for x in (pi, mu, act, rew, disc, val)] for _ in range(nsets)]
    outs = [[hip.DeviceBuffer(n) for n in (T * B * 4, T * B * 4, T * B * A * 4, (T + 1) * B * 4, 24)]
            for _ in range(nsets)]
    H = _abi.VtraceHparams(rho_bar=1.0, c_bar=1.0, pg_rho_bar=1.0, lambda_=1.0,
                           baseline_cost=0.5, entropy_cost=0.01)
    ref = None
    for path in libs:
      for variant in (args.variant or [0]):
        L = _abi.lib() if path is None else C.CDLL(os.path.abspath(path))
        if path is not None:
            for name, (argt, res) in _abi.SIGNATURES.items():
                if hasattr(L, name):
                    f = getattr(L, name)
                    f.restype, f.argtypes = res, argt
        wsb = L.fi_vtrace_workspace_bytes(T, B, A)
        wss = [hip.DeviceBuffer(wsb) for _ in range(nsets)]
        for w in wss:
            w.zero()

        def launch(i):
            k = i % nsets
            rc = L.fi_vtrace_loss_fp32_variant(variant, T, B, A, *[b.ptr for b in bufs[k]], C.byref(H),
                                               *[o.ptr for o in outs[k]], wss[k].ptr, wsb, None)
            assert rc == 0, rc

        for i in range(max(5, nsets)):
            launch(i)
        e0, e1 = hip.Event(), hip.Event()
        e0.record()
        for i in range(args.iters):
            launch(i)
        e1.record()
        hip.synchronize()
        ms = e0.elapsed_ms(e1) / args.iters
        gbs = (12 * A + 28) * T * B / (ms * 1e-3) / 1e9
        dl = outs[0][2].download(np.float32, (T, B, A))
        diff = 0.0 if ref is None else float(np.abs(dl - ref).max())
        ref = dl if ref is None else ref
        print(f"{path or 'default'} variant {variant} sets {nsets}: {ms * 1e3:.2f} us/launch  {gbs:.0f} GB/s  "
              f"({gbs / 8000:.1%} of 8 TB/s)  max|d dlogits| vs first {diff:.2e}", flush=True)
        ws = wss[0]
        if args.stamps and wsb >= 8 * (1024 + (B // 8) * 20):
            nblk = B // 8
            st = ws.download(np.uint64, (wsb // 8,))[1024:1024 + nblk * 20].reshape(nblk, 20)
            st = st.astype(np.int64)
            n = int((st[0] > 0).sum())
            t = (st[:, :n] - st[:, :1].min()) * 10 / 1000.0  # us (100 MHz)
            names = ["start"] + [f"{p}{k}" for k in range((n - 2) // 4) for p in ("B1_", "iss", "B2_", "end")] + ["done"]
            for j in range(n):
                q = np.percentile(t[:, j], [0, 50, 100])
                print(f"  {names[j] if j < len(names) else j:>6}: min {q[0]:6.2f}  med {q[1]:6.2f}  max {q[2]:6.2f} us")


if __name__ == "__main__":
    main()
