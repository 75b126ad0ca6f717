import os, sys
R = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, R); sys.path.insert(0, os.path.join(R, "monodepth2.jl_amd"))
import torch
from tests import _data as D
from tests._model_parity import run
modes = sys.argv[1:] or ["both"]
for strict in ((True, False) if "both" in modes else (True,)):
    g, o, errs = run(strict=strict)
    print("strict", strict, "loss", g["loss"], g["tail_loss"], o["loss"])
    print(" disp rel", [D.rel_err(a, b) for a, b in zip(g["disps"], o["disps"])], "pose rel", D.rel_err(g["pose"], o["pose"]))
    print(" total grad rel", D.rel_err(g["grad"], o["grad"]))
    groups = {}
    for k, v in errs.items():
        grp = ".".join(k.split(".")[:2])
        groups[grp] = max(groups.get(grp, 0.0), v)
    for k, v in groups.items(): print(f"   {k:30s} {v:.3e}")
    worst = sorted(errs.items(), key=lambda kv: -kv[1])[:12]
    for k, v in worst: print(f"   {k:40s} {v:.3e}")
