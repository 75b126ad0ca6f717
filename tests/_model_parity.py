"""Full train-step parity helper: GPU Model (libmd2hip) vs the fp64 CPU oracle on the same
flat parameters and inputs, with the GPU's per-pixel argmin imposed on the oracle."""
import torch

import md2hip
from oracle import md2_oracle as O
from tests import _data as D


DEFAULT_SCALES = {1: 0.0625, 2: 0.125, 3: 0.25, 4: 0.5, 5: 1.0}


def run(N=2, C=3, H=64, W=128, arch=18, strict=True, seed=7, automasking=False, levels=(2, 3, 4, 5),
        target_id=2, source_ids=(1, 3)):
    x = D.triplets(N, C, H, W, seed=seed, ramp_sources=strict)
    K, invK = D.intrinsics(W, H)
    enc = md2hip.ResNet(arch, in_channels=C)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=list(levels),
                                                  embedding_levels=0),
                         md2hip.PoseDecoder(enc.stages[-1]), seed=42)
    scales = tuple(DEFAULT_SCALES[l] for l in levels)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), target_id=target_id,
                              source_ids=tuple(source_ids), scales=scales)
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=automasking)
    xg = x.float().cuda().contiguous()
    loss, *_ = md2hip.train_loss(model, xg, None, cache, params)
    disps, pose = model._last.outputs()
    md2hip.gradient(model)
    poses_g = [(pose[:N, :3].contiguous(), pose[:N, 3:].contiguous()),
               (pose[N:, :3].contiguous(), pose[N:, 3:].contiguous())]
    tail = md2hip.loss_tail([d.contiguous() for d in disps], poses_g, xg, None, cache, params, visualize=True)
    torch.cuda.synchronize()
    g = {"loss": loss.item(), "tail_loss": tail["loss"].item(), "disps": [d.cpu() for d in disps],
         "pose": pose.cpu(), "grad": model.grad.cpu(), "sel": tail["vis_sel"].cpu(),
         "flat": model.flat.detach().double().cpu()}
    g["decisions"] = gpu_decisions(model, N, arch, target_id=target_id, source_ids=source_ids)
    spec = O.param_spec(arch, C, tuple(levels))
    flat = model.flat.detach().double().cpu().clone().requires_grad_(True)
    P = O.unflatten(flat, spec)
    with O.forced_decisions(g["decisions"]):
        d_o, p_o = O.model_forward(P, x, source_ids, target_id, arch=arch, scale_levels=tuple(levels))
    cache_o = O.TrainCache(K=K, invK=invK, target_id=target_id, source_ids=tuple(source_ids), scales=scales)
    par_o = O.Params(target_size=(W, H), batch_size=N, automasking=automasking)
    # the GPU's argmin (-1 = automask) as an index into [auto_loss?, source 0, source 1]
    forced = [g["sel"][s].unsqueeze(1).long() + (1 if automasking else 0) for s in range(len(levels))]
    auto_o = O.automasking_loss(x, x[:, target_id - 1], source_ids) if automasking else None
    loss_o = O.loss_from_outputs(d_o, p_o, x, auto_o, cache_o, par_o, forced_sel=forced)
    loss_o.backward()
    o = {"loss": loss_o.item(), "disps": [d.detach() for d in d_o],
         "pose": torch.cat([torch.cat([r, t], 1) for r, t in p_o], 0).detach(), "grad": flat.grad}
    errs = {}
    for name, shape, off in [(n, s, None) for n, s in spec]:
        pass
    off = 0
    for name, shape in spec:
        n = 1
        for s in shape:
            n *= s
        errs[name] = D.rel_err(g["grad"][off:off + n], o["grad"][off:off + n])
        off += n
    return g, o, errs


def gpu_decisions(model, N, arch=18, L=3, target_id=2, source_ids=(1, 3)):
    """The GPU forward's branch decisions (ReLU masks, max-pool argmax) in the oracle's layout
    (encoder batch n-major; pose per source pair) for O.forced_decisions."""
    from oracle import md2_oracle as O
    t = {k: v.cpu() for k, v in model._last.debug_tensors().items()}

    def nmajor(v):   # frame-major [L*N, ...] -> n-major [N*L, ...]
        return v.reshape(L, N, *v.shape[1:]).transpose(0, 1).reshape(L * N, *v.shape[1:])

    d = {"stem": nmajor(t["stem.out"] > 0), "maxpool": nmajor(t["maxpool.arg"])}
    for si, nb in enumerate(O.RESNET_LAYERS[arch]):
        for bi in range(nb):
            q = f"layer{si + 1}.{bi}"
            d[f"encoder.{q}.out"] = nmajor(t[q + ".out"] > 0)
            for r in ("relu1", "relu2"):           # BasicBlock: relu1; Bottleneck: relu1, relu2
                if f"{q}.{r}" in t:
                    d[f"encoder.{q}.{r}"] = nmajor(t[f"{q}.{r}"] > 0)
    sq = t["pose.sq"] > 0                    # squeezer outputs of the 3N frame-major images
    for j, s in enumerate(source_ids):       # pair j = frames (min(s,t), max(s,t)), GPU rows [jN, (j+1)N)
        a, b = min(s, target_id) - 1, max(s, target_id) - 1
        d[f"pose{j}.sqa"] = sq[a * N:(a + 1) * N]
        d[f"pose{j}.sqb"] = sq[b * N:(b + 1) * N]
        d[f"pose{j}.conv1"] = t["pose.conv1"][j * N:(j + 1) * N] > 0
        d[f"pose{j}.conv2"] = t["pose.conv2"][j * N:(j + 1) * N] > 0
    return d


def oracle_at_gpu_outputs(g, N=2, C=3, H=64, W=128, arch=18, strict=True, seed=7):
    """The fp64 oracle's gradient with the loss tail evaluated AT THE GPU's forward outputs
    (disparities, poses) and back-propagated through the oracle's own networks (value substituted,
    graph kept: d_o + (d_gpu - d_o).detach()).  Against the plain oracle this isolates how much
    of a gradient difference the ~1e-6 forward discrepancy alone explains; against the GPU it
    measures the backward's own accuracy."""
    x = D.triplets(N, C, H, W, seed=seed, ramp_sources=strict)
    K, invK = D.intrinsics(W, H)
    spec = O.param_spec(arch, C, (2, 3, 4, 5))
    f = g["flat"].double().clone().requires_grad_(True)
    P = O.unflatten(f, spec)
    with O.forced_decisions(g["decisions"]):
        d_o, p_o = O.model_forward(P, x, arch=arch)
    d_s = [d + (dg.double().view_as(d) - d).detach() for d, dg in zip(d_o, g["disps"])]
    pg = g["pose"].double()
    p_s = []
    for k, (r, t) in enumerate(p_o):
        q = pg[k * N:(k + 1) * N]
        p_s.append((r + (q[:, :3] - r).detach(), t + (q[:, 3:] - t).detach()))
    cache_o = O.TrainCache(K=K, invK=invK)
    par_o = O.Params(target_size=(W, H), batch_size=N, automasking=False)
    forced = [s.unsqueeze(1).long() for s in g["sel"]]
    O.loss_from_outputs(d_s, p_s, x, None, cache_o, par_o, forced_sel=forced).backward()
    return f.grad.double()


def oracle_fp32_floor(N=2, C=3, H=64, W=128, arch=18, strict=True, seed=7, flat=None, sel=None,
                      decisions=None, levels=(2, 3, 4, 5), target_id=2, source_ids=(1, 3)):
    """Per-tensor gradient error of the SAME oracle run in fp32 vs fp64 (the fp32 noise floor),
    plus the forward outputs' floors under the keys "__disp<s>" and "__pose"."""
    x = D.triplets(N, C, H, W, seed=seed, ramp_sources=strict)
    K, invK = D.intrinsics(W, H)
    spec = O.param_spec(arch, C, tuple(levels))
    scales = tuple(DEFAULT_SCALES[l] for l in levels)
    grads, fwd, losses = [], [], []
    for dt in (torch.float64, torch.float32):
        f = flat.to(dt).clone().requires_grad_(True)
        P = O.unflatten(f, spec)
        with O.forced_decisions(decisions or {}):
            d_o, p_o = O.model_forward(P, x.to(dt), source_ids, target_id, arch=arch,
                                       scale_levels=tuple(levels))
        fwd.append(([d.detach().double() for d in d_o],
                    torch.cat([torch.cat([r, t], 1) for r, t in p_o], 0).detach().double()))
        cache_o = O.TrainCache(K=K.to(dt), invK=invK.to(dt), target_id=target_id,
                               source_ids=tuple(source_ids), scales=scales)
        par_o = O.Params(target_size=(W, H), batch_size=N, automasking=False)
        forced = [s.unsqueeze(1).long() for s in sel]
        lo = O.loss_from_outputs(d_o, p_o, x.to(dt), None, cache_o, par_o, forced_sel=forced)
        lo.backward()
        losses.append(lo.item())
        grads.append(f.grad.double())
    errs, off = {}, 0
    for name, shape in spec:
        n = 1
        for s in shape:
            n *= s
        errs[name] = D.rel_err(grads[1][off:off + n], grads[0][off:off + n])
        off += n
    # forward outputs: "__disp<s>" per scale and "__pose"
    for s_, (a, b) in enumerate(zip(fwd[1][0], fwd[0][0])):
        errs[f"__disp{s_}"] = D.rel_err(a, b)
    errs["__pose"] = D.rel_err(fwd[1][1], fwd[0][1])
    errs["__loss"] = abs(losses[1] - losses[0]) / abs(losses[0])
    return errs
