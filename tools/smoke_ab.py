"""smoke()'s model-parity case (N=1, 64x128) printing the GPU and oracle losses, the disparity /
pose errors and the worst per-tensor gradient errors -- for comparing kernel switches
(MD2_TUNING=1 ...)."""
import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [R, os.path.join(R, "monodepth2.jl_amd")]
import torch
from tests import _data as D
from tests._model_parity import run
torch.cuda.set_device(0)
g, o, errs = run(N=1, H=64, W=128, strict=True)
w = sorted(errs.items(), key=lambda kv: -kv[1])[:3]
de = [f"{D.rel_err(a, b):.1e}" for a, b in zip(g["disps"], o["disps"])]
tag = " ".join(f"{k}={v}" for k, v in os.environ.items() if k.startswith("MD2_")) or "default"
print(tag, f"| gpu {g['loss']:.9f} oracle {o['loss']:.9f} tail {g['tail_loss']:.9f} | disp {de} pose "
      f"{D.rel_err(g['pose'], o['pose']):.1e} |", [(k, f"{v:.1e}") for k, v in w])
