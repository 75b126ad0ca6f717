"""Full-step parity diagnostics: the worst per-tensor gradient errors of the GPU step against the
fp64 oracle with the GPU's decisions imposed (tests/_model_parity.py), plus the fp32 floor.
usage: python tools/model_diag.py [strict 0/1] [N] [H] [W]"""
import os
import sys

R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R)
sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
from tests._model_parity import oracle_fp32_floor, run  # noqa: E402

strict = (sys.argv[1] != "0") if len(sys.argv) > 1 else False
N = int(sys.argv[2]) if len(sys.argv) > 2 else 2
H = int(sys.argv[3]) if len(sys.argv) > 3 else 64
W = int(sys.argv[4]) if len(sys.argv) > 4 else 128
g, o, errs = run(N=N, H=H, W=W, strict=strict)
floor = oracle_fp32_floor(N=N, H=H, W=W, strict=strict, flat=g["flat"], sel=[s for s in g["sel"]],
                          decisions=g["decisions"])
print(f"loss gpu {g['loss']:.9f} oracle {o['loss']:.9f} rel {abs(g['loss'] - o['loss']) / o['loss']:.2e}")
for k, v in sorted(errs.items(), key=lambda kv: -kv[1])[:10]:
    print(f"  {k:32s} {v:.3e}  (fp32 floor {floor[k]:.2e})")
from tests._model_parity import oracle_at_gpu_outputs  # noqa: E402
from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402
sub = oracle_at_gpu_outputs(g, N=N, H=H, W=W, strict=strict)
off = 0
rows = []
for name, shape in O.param_spec(18, 3, (2, 3, 4, 5)):
    n = 1
    for s_ in shape:
        n *= s_
    rows.append((name, D.rel_err(g["grad"][off:off + n], sub[off:off + n]),
                 D.rel_err(sub[off:off + n], o["grad"][off:off + n])))
    off += n
print("GPU vs oracle-at-GPU-outputs (backward accuracy) | oracle-at-GPU-outputs vs oracle (forward discrepancy):")
for name, e1, e2 in sorted(rows, key=lambda r: -r[1])[:8]:
    print(f"  {name:32s} {e1:.3e} | {e2:.3e}")
print("  head2.bias:", [f"{e1:.2e} | {e2:.2e}" for n_, e1, e2 in rows if n_ == "depth.head2.bias"])
