"""Per-workgroup phase timeline of the Winograd PRE conv (wino_f23_k16_kernel<true> where
Cout % 128 == 0 and Cin % 16 == 0; diagnostic).

Loads lib/libbpk_wino_timing.so (conv_winograd.hip built with -DWINO_TIMING: each workgroup
records the 100 MHz wall clock at entry, after its prologue, after its chunk loop and after
its epilogue, plus the CU it ran on) and runs the PRE+stats conv of the given shapes.
Reports per-workgroup phase durations and, per CU, the idle gap between one workgroup's
end and the next one's start, and how many workgroups were resident on a CU at once.
Usage: python tools/wino_timing.py [cin cout hw] ...  (default: the 128->128@128 and
256->256@128 shapes of the NCSN++ mix, B=64)
"""
import ctypes
import os
import sys

import numpy as np
import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB = os.environ.get("WINO_TIMING_LIB", os.path.join(REPO, "b-pinn-kalman-filter_amd", "lib",
                                                    "libbpk_wino_timing.so"))
TICK_US = 0.01  # wall_clock64: 100 MHz


def run(lib, B, cin, cout, hw, dev):
    g = torch.Generator(device=dev).manual_seed(0)
    x = torch.randn(B, cin, hw, hw, device=dev, generator=g)
    w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
    b = torch.randn(cout, device=dev, generator=g)
    pre = torch.stack([torch.rand(B, cin, device=dev, generator=g) + 0.5,
                       torch.randn(B, cin, device=dev, generator=g) * 0.1], -1).contiguous()
    nU = lib.bpk_conv3x3_wino_filter_bytes(cin, cout) // 4
    U = torch.empty(nU, device=dev)
    y = torch.empty(B, cout, hw, hw, device=dev)
    R = (hw // 8) * (hw // 16)
    part = torch.empty(B, cout, R, 2, device=dev)
    P = ctypes.c_void_p
    assert lib.bpk_conv3x3_wino_filter_f32(P(w.data_ptr()), P(U.data_ptr()), cin, cout, None) == 0

    def call():
        rc = lib.bpk_conv3x3_wino_ex_f32(P(x.data_ptr()), None, cin, P(pre.data_ptr()),
                                         P(U.data_ptr()), P(b.data_ptr()), None,
                                         ctypes.c_float(1.0), P(y.data_ptr()),
                                         P(part.data_ptr()), B, cin, cout, hw, hw, None)
        assert rc == 0, lib.bpk_last_error()
    for _ in range(int(os.environ.get("WINO_TIMING_WARM", "30"))):  # clocks ramp up
        call()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    call()
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e)
    nblk = B * (hw // 16) * (hw // 8) * ((cout + 63) // 64)
    if cout % 128 == 0:
        nblk //= 2  # 8-wave forms: 128 couts per workgroup (no split-K at these B = 64 shapes)
    ts6 = np.zeros((nblk, 8), dtype=np.int64)
    cu = np.zeros(nblk, dtype=np.uint32)
    n = lib.bpk_wino_timing_read(ts6.ctypes.data_as(P), cu.ctypes.data_as(P), nblk)
    assert n == nblk, n
    ts = ts6[:, [0, 3, 4, 5]]
    ghz = (ts6[:, 7] - ts6[:, 6]) / ((ts6[:, 5] - ts6[:, 0]) * TICK_US * 1e3)
    sub = (ts6[:, 1:4] - ts6[:, 0:3]) * TICK_US
    print(f"  prologue parts us (mean): loads landed {sub[:, 0].mean():.2f}, patch stores "
          f"{sub[:, 1].mean():.2f}, first transform {sub[:, 2].mean():.2f}")
    t0 = ts[:, 0].min()
    t = (ts - t0) * TICK_US  # us
    pro, loop, epi = t[:, 1] - t[:, 0], t[:, 2] - t[:, 1], t[:, 3] - t[:, 2]
    span = t[:, 3].max()
    fl = 2.0 * B * cin * cout * 16 * (hw // 2) ** 2
    print(f"== {cin}->{cout}@{hw} B={B}: {nblk} workgroups, event {ms:.3f} ms, "
          f"timeline span {span / 1e3:.3f} ms, {fl / ms / 1e9:.1f} TFLOP/s executed; shader clock "
          f"{np.median(ghz):.3f} GHz (p10 {np.percentile(ghz, 10):.3f}, p90 {np.percentile(ghz, 90):.3f})")
    for name, v in (("prologue", pro), ("loop", loop), ("epilogue", epi), ("total", t[:, 3] - t[:, 0])):
        print(f"  {name:9s} us: mean {v.mean():7.2f}  p10 {np.percentile(v, 10):7.2f}  "
              f"p50 {np.percentile(v, 50):7.2f}  p90 {np.percentile(v, 90):7.2f}  max {v.max():7.2f}")
    # per CU: sort by start; residency and gaps
    ucu = np.unique(cu)
    gaps, occ_hist, first = [], np.zeros(8), []
    for c in ucu:
        idx = np.where(cu == c)[0]
        st, en = t[idx, 0], t[idx, 3]
        o = np.argsort(st)
        st, en = st[o], en[o]
        first.append(st[0])
        # events sweep: residency over time
        ev = sorted([(a, 1) for a in st] + [(b_, -1) for b_ in en])
        cur, last = 0, ev[0][0]
        for tt, d in ev:
            occ_hist[min(cur, 7)] += tt - last
            cur += d
            last = tt
        # each start after the first two: gap from the latest end before it
        for i in range(len(st)):
            prev_end = en[:i][en[:i] <= st[i]]
            if len(prev_end):
                gaps.append(st[i] - prev_end.max())
    gaps = np.array(gaps)
    occ = occ_hist / occ_hist.sum()
    print(f"  {len(ucu)} CUs seen; workgroups per CU {nblk / len(ucu):.1f}; "
          f"time at residency 0/1/2/3: {occ[0]:.3f} {occ[1]:.3f} {occ[2]:.3f} {occ[3]:.3f}")
    if len(gaps):
        print(f"  start gap after a resident wg ended, us: mean {gaps.mean():.2f} p50 "
              f"{np.percentile(gaps, 50):.2f} p90 {np.percentile(gaps, 90):.2f}")
    fs = np.array(first)
    print(f"  first start per CU, us: p50 {np.percentile(fs, 50):.2f} max {fs.max():.2f}; "
          f"last end p10 {np.percentile(t[:, 3], 99.9):.1f}")
    # phase alignment of co-resident pairs: |start difference| of workgroups whose spans overlap
    return dict(shape=f"{cin}->{cout}@{hw}", ms=ms, pro=float(pro.mean()), loop=float(loop.mean()),
                epi=float(epi.mean()), occ=occ[:4].tolist(), gap=float(gaps.mean()) if len(gaps) else None)


def main():
    dev = torch.device("cuda:0")
    torch.cuda.init()
    lib = ctypes.CDLL(LIB, mode=ctypes.RTLD_GLOBAL)
    lib.bpk_conv3x3_wino_filter_bytes.restype = ctypes.c_int64
    lib.bpk_last_error.restype = ctypes.c_char_p
    a = [int(v) for v in sys.argv[1:]]
    shapes = [tuple(a[i:i + 3]) for i in range(0, len(a), 3)] or [(128, 128, 128), (256, 256, 128),
                                                                  (256, 256, 32)]
    for cin, cout, hw in shapes:
        run(lib, 64, cin, cout, hw, dev)


if __name__ == "__main__":
    main()
