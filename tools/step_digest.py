"""Bit-identity digest of the bench train step: `steps` full steps (forward + loss + backward +
ADAM) at B, 416x128 on the bench's synthetic batch, then SHA-256 of the loss, the flat
parameters and the flat gradient.  Run it once per library (MD2HIP_LIB=...) to show that a
kernel change only regroups work (same digest) or to see that it re-rounds (different digest).

    python tools/step_digest.py [B] [steps]"""
import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "monodepth2.jl_amd")]


def main():
    B = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    import torch
    import md2hip
    import md2hip.dist
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    enc = md2hip.ResNet(18, in_channels=3)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=[2, 3, 4, 5],
                                                  embedding_levels=0),
                         md2hip.PoseDecoder(512), device=dev, seed=42)
    K, invK = md2hip.depth10k_intrinsics(416, 128)
    cache = md2hip.TrainCache(K=K, invK=invK, scales=(0.125, 0.25, 0.5, 1.0))
    params = md2hip.Params(target_size=(416, 128), batch_size=B, automasking=False, disparity_smoothness=1e-3)
    opt = md2hip.ADAM(1e-4)
    x = md2hip.dist.synthetic_triplets(B, 128, 416, 0, dev)
    ex = model.executor(tuple(x.shape), cache, params)
    loss = torch.empty(1, dtype=torch.float32, device=dev)
    losses = []
    for _ in range(steps):
        md2hip.dist.train_step(ex, model, opt, x, loss=loss)
        torch.cuda.synchronize()
        losses.append(loss.item())

    def h(t):
        return hashlib.sha256(t.detach().cpu().numpy().tobytes()).hexdigest()[:16]
    print(json.dumps({"lib": os.environ.get("MD2HIP_LIB", "default"), "B": B, "steps": steps,
                      "losses": losses, "params": h(model.flat), "grad": h(model.grad)}))


if __name__ == "__main__":
    main()
