"""The Winograd conv with the GroupNorm+SiLU prologue (wino_f23_pipe_kernel<1, true>, the
sampler's dominant kernel) over the NCSN++ 128x128 shape mix, B = 64: per shape the PRE
form with bias + GroupNorm partial statistics (Conv_0 of a BigGAN block) and with the
residual tail (Conv_1), each weighted by its count per forward (SURVEY 8(a) a11 inventory).
Prints one JSON line per shape and a weighted summary.  BPK_LIB selects the library."""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch  # noqa: E402

from op.conv import conv3x3, filter_transform  # noqa: E402

# (cin, cout, hw, PRE+stats convs per forward, PRE+residual convs per forward)
from bench import WINO_MIX as MIX  # noqa: E402  (the census of one forward)
B = int(os.environ.get("B", 64))
REPS = int(os.environ.get("REPS", 10))


def t_of(fn, st):
    with torch.cuda.stream(st):
        for _ in range(3):
            fn()
        s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        s.record(st)
        for _ in range(REPS):
            fn()
        e.record(st)
    e.synchronize()
    return s.elapsed_time(e) / REPS / 1e3


def main():
    dev = torch.device("cuda:0")
    st = torch.cuda.Stream(dev)
    g = torch.Generator(device=dev).manual_seed(0)
    tot_t = tot_f = 0.0
    for cin, cout, hw, n_pre, n_res in MIX:
        x = torch.randn(B, cin, hw, hw, device=dev, generator=g)
        w = torch.randn(cout, cin, 3, 3, device=dev, generator=g) / (3 * cin ** 0.5)
        b = torch.randn(cout, device=dev, generator=g)
        pre = torch.stack([torch.rand(B, cin, device=dev, generator=g) + 0.5,
                           torch.randn(B, cin, device=dev, generator=g) * 0.1], -1).contiguous()
        skip = torch.randn(B, cout, hw, hw, device=dev, generator=g)
        filter_transform(w)
        t_pre = t_of(lambda: conv3x3(x, w, b, pre=pre, stats=True), st)
        t_res = t_of(lambda: conv3x3(x, w, b, skip=skip, div=2 ** 0.5, pre=pre, stats=True), st)
        fl = 2.0 * B * cin * cout * 16 * (hw // 2) ** 2  # executed (Winograd) MFMA FLOPs
        tot_t += n_pre * t_pre + n_res * t_res
        tot_f += (n_pre + n_res) * fl
        print(json.dumps(dict(shape=f"{cin}->{cout}@{hw}", pre_ms=round(t_pre * 1e3, 4),
                              res_ms=round(t_res * 1e3, 4),
                              pre_tflops=round(fl / t_pre / 1e12, 1),
                              res_tflops=round(fl / t_res / 1e12, 1))), flush=True)
    print(json.dumps(dict(summary="weighted mix", lib=os.environ.get("BPK_LIB", "default"),
                          ms_per_forward_mix=round(tot_t * 1e3, 3),
                          tflops_executed=round(tot_f / tot_t / 1e12, 2),
                          frac_of_157_3=round(tot_f / tot_t / 1e12 / 157.3, 4))), flush=True)


if __name__ == "__main__":
    main()
