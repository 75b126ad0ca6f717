"""Decompose a GPU train step's gradient error (tools/model_dump.py file) into
  tail:     the GPU loss tail's d_disp / d_pose vs the fp64 oracle tail evaluated AT the GPU's own
            disparities / poses (decisions imposed) -- and the fp32 oracle's error for scale,
  networks: the GPU flat gradient vs the fp64 oracle networks' backward driven by the GPU's OWN
            tail cotangents (forward decisions imposed) -- the decoder / encoder backward alone.
    python tools/model_analyze.py DUMP.pt"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]
import torch  # noqa: E402

from oracle import md2_oracle as O  # noqa: E402
from tests import _data as D  # noqa: E402
from tests._model_parity import per_tensor  # noqa: E402

torch.set_num_threads(min(16, os.cpu_count()))
dmp = torch.load(sys.argv[1], weights_only=False)
g = dmp["g"]
x = g["x"]
N, L, C, H, W = x.shape
K, invK = D.intrinsics(W, H)
sel = [s.unsqueeze(1).long() for s in g["sel"]]


def tail(dt):
    ds = [d.to(dt).clone().requires_grad_(True) for d in g["disps"]]
    p = g["pose"].to(dt)
    ps = [(p[k * N:(k + 1) * N, :3].clone().requires_grad_(True), p[k * N:(k + 1) * N, 3:].clone().requires_grad_(True))
          for k in range(2)]
    l = O.loss_from_outputs(ds, ps, x.to(dt), None, O.TrainCache(K=K.to(dt), invK=invK.to(dt)),
                            O.Params(target_size=(W, H), batch_size=N, automasking=False),
                            forced_sel=sel, forced_cells=g["cells"])
    l.backward()
    return [d.grad.double() for d in ds], torch.cat([torch.cat([r.grad, t.grad], 1) for r, t in ps]).double()


d64, p64 = tail(torch.float64)
d32, p32 = tail(torch.float32)
for s in range(len(d64)):
    print(f"tail scale {s}: gpu {D.rel_err(g['tail_d_disp'][s], d64[s]):.2e}   fp32-oracle {D.rel_err(d32[s], d64[s]):.2e}")
print(f"tail d_pose: gpu {D.rel_err(g['tail_d_pose'], p64):.2e}   fp32-oracle {D.rel_err(p32, p64):.2e}")

# networks driven by the GPU's own tail cotangents
spec = O.param_spec(18, C, (2, 3, 4, 5))
for name, dd, dp in (("gpu-cotangents", g["tail_d_disp"], g["tail_d_pose"]), ("oracle-cotangents", d64, p64)):
    f = g["flat"].double().clone().requires_grad_(True)
    P = O.unflatten(f, spec)
    with O.forced_decisions(g["decisions"]):
        do, po = O.model_forward(P, x)
    tot = sum((a * b.double()).sum() for a, b in zip(do, dd))
    pp = torch.cat([torch.cat([r, t], 1) for r, t in po], 0)
    tot = tot + (pp * dp.double()).sum()
    tot.backward()
    e = per_tensor(spec, g["grad"], f.grad)
    worst = sorted(e.items(), key=lambda kv: -kv[1])[:6]
    print(f"networks vs oracle backward from {name}: " + ", ".join(f"{k} {v:.2e}" for k, v in worst))
print("end-to-end (test):", ", ".join(f"{k} {v:.2e}" for k, v in sorted(dmp["errs"].items(), key=lambda kv: -kv[1])[:6]))
