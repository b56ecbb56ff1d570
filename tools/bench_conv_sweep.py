"""Winograd conv3x3 time vs Cin (Cout = 128 @64^2, B = 64): separates the per-workgroup fixed
cost (prologue / epilogue, in chunk-equivalents) from the per-chunk main-loop cost; plain and
GroupNorm-prologue (pre=) forms."""
import json, os, sys
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(REPO, "b-pinn-kalman-filter_amd"), REPO]
import torch
from op.conv import conv3x3, filter_transform
dev = torch.device("cuda:0")
B = int(os.environ.get("B", 64))
def t_of(fn, reps=10):
    for _ in range(3): fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps): fn()
    e.record(); e.synchronize()
    return s.elapsed_time(e) / reps / 1e3
for cin in (32, 64, 128, 256, 512, 1024):
  for hw in (64, 128):
      if hw == 128 and cin > 256: continue
      x = torch.randn(B, cin, hw, hw, device=dev)
      w = torch.randn(128, cin, 3, 3, device=dev) / (3 * cin ** 0.5)
      pre = torch.stack([torch.rand(B, cin, device=dev) + 0.5, torch.randn(B, cin, device=dev)], -1)
      filter_transform(w)
      t = t_of(lambda: conv3x3(x, w))
      tp = t_of(lambda: conv3x3(x, w, pre=pre))
      fl = 2.0 * B * cin * 128 * 9 * hw * hw
      print(json.dumps(dict(cin=cin, hw=hw, ms=round(t * 1e3, 4), ms_pre=round(tp * 1e3, 4),
                            tflops_eff=round(fl / t / 1e12, 1), tflops_eff_pre=round(fl / tp / 1e12, 1))),
            flush=True)
