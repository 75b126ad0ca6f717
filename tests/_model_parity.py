"""Full train-step parity helper: GPU Model (libmd2hip) vs the fp64 CPU oracle on the same
flat parameters and inputs, with the GPU's branch decisions imposed on the oracle.

The objective is piecewise smooth.  Its branch decisions are: the per-pixel argmin over sources
(src/training.jl:13-15), ReLU masks and max-pool argmax (encoder / pose decoder), and grid_sample's
bilinear cell and border clamp (src/training.jl:56).  A decision whose inputs sit within fp32
rounding of its switching point flips between the fp32 GPU and the fp64 oracle, and one flipped
decision moves the gradient by O(1) at that pixel.  Each decision the GPU made is therefore
recorded (``vis_sel``, ``vis_cell``, ``md2_model_debug_tensor``) and imposed on the oracle
(``forced_sel``, ``forced_cells``, ``O.forced_decisions``); the oracle then evaluates the same
smooth function as the GPU, and the comparison is pure fp32-vs-fp64 accuracy.

Source frames (``sources``):
  "ramp"     affine ramps (bilinear sampling of them has no kinks at all),
  "texture"  low-frequency texture + 15 % pixel noise (tests/_data.py),
  "uniform"  the bench's own i.i.d. U[0,1) triplets (md2hip.dist.synthetic_triplets)."""
import torch

import md2hip
from oracle import md2_oracle as O
from tests import _data as D


DEFAULT_SCALES = {1: 0.0625, 2: 0.125, 3: 0.25, 4: 0.5, 5: 1.0}


def inputs(N, C, H, W, sources="ramp", seed=7):
    if sources == "uniform":
        from md2hip.dist import synthetic_triplets
        return synthetic_triplets(N, H, W, 0, "cpu", channels=C).double()
    return D.triplets(N, C, H, W, seed=seed, ramp_sources=(sources == "ramp"))


def _sources(strict, sources):
    return sources if sources is not None else ("ramp" if strict else "texture")


def mpi_bins(N, num_bins, seed=3):
    """Seeded disparity bins (the reference's CUDA.rand draw injected, defect D3)."""
    u = torch.rand(N, num_bins, generator=torch.Generator().manual_seed(seed), dtype=torch.float64)
    return md2hip.disparity_bins(N, num_bins, u=u, device="cpu")


def run(N=2, C=3, H=64, W=128, arch=18, strict=True, seed=7, automasking=False, levels=(2, 3, 4, 5),
        target_id=2, source_ids=(1, 3), sources=None, num_bins=0):
    """num_bins > 0: the MPI-mode Model (DepthDecoder(embedding_levels=21), batch 1, num_bins
    planes) against O.mpi_train_loss."""
    sources = _sources(strict, sources)
    x = inputs(N, C, H, W, sources, seed)
    K, invK = D.intrinsics(W, H)
    emb = 21 if num_bins else 0
    enc = md2hip.ResNet(arch, in_channels=C)
    model = md2hip.Model(enc, md2hip.DepthDecoder(encoder_channels=enc.stages, scale_levels=list(levels),
                                                  embedding_levels=emb),
                         md2hip.PoseDecoder(enc.stages[-1]), seed=42)
    scales = tuple(DEFAULT_SCALES[l] for l in levels)
    cache = md2hip.TrainCache(K=K.numpy(), invK=invK.numpy(), target_id=target_id,
                              source_ids=tuple(source_ids), scales=scales)
    params = md2hip.Params(target_size=(W, H), batch_size=N, automasking=automasking)
    xg = x.float().cuda().contiguous()
    bins = mpi_bins(N, num_bins) if num_bins else None
    nb = max(1, num_bins)
    loss, *_ = md2hip.train_loss(model, xg, None, cache, params, num_bins=nb,
                                 bins=bins.cuda() if bins is not None else None)
    disps, pose = model._last.outputs()
    md2hip.gradient(model)
    # the loss tail again at the GPU's outputs, recording its argmin and bilinear cells (planes of
    # an MPI sample broadcast its frames and poses: repeated here)
    xt = xg.repeat_interleave(nb, 0).contiguous() if nb > 1 else xg
    poses_g = [(pose[s * N:(s + 1) * N, :3].repeat_interleave(nb, 0).contiguous(),
                pose[s * N:(s + 1) * N, 3:].repeat_interleave(nb, 0).contiguous()) for s in range(2)]
    params_t = md2hip.Params(target_size=(W, H), batch_size=N * nb, automasking=automasking)
    am_t = None
    if automasking:
        from md2hip.primitives import automasking_loss
        am_t = automasking_loss(xg, target_id, tuple(source_ids)).repeat_interleave(nb, 0).contiguous()
    tail = md2hip.loss_tail([d.contiguous() for d in disps], poses_g, xt, am_t, cache, params_t, visualize=True)
    torch.cuda.synchronize()
    g = {"loss": loss.item(), "tail_loss": tail["loss"].item(), "disps": [d.cpu() for d in disps],
         "pose": pose.cpu(), "grad": model.grad.cpu(), "sel": tail["vis_sel"].cpu(),
         "cells": tail["vis_cell"].cpu(), "flat": model.flat.detach().double().cpu(),
         "x": x, "sources": sources, "automasking": automasking, "bins": bins,
         "levels": tuple(levels), "target_id": target_id, "source_ids": tuple(source_ids)}
    g["decisions"] = gpu_decisions(model, N, arch, target_id=target_id, source_ids=source_ids)
    grad_o, fwd_o, loss_o, spec = _oracle_grad(g, torch.float64, arch, levels, target_id, source_ids)
    o = {"loss": loss_o, "disps": fwd_o[0], "pose": fwd_o[1], "grad": grad_o}
    return g, o, per_tensor(spec, g["grad"], o["grad"])


def per_tensor(spec, a, b):
    errs, off = {}, 0
    for name, shape in spec:
        n = 1
        for s in shape:
            n *= s
        errs[name] = D.rel_err(a[off:off + n], b[off:off + n])
        off += n
    return errs


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


def _oracle_grad(g, dt, arch, levels, target_id, source_ids, perturb=None, seed=0):
    """The oracle's flat gradient in dtype ``dt`` with every GPU decision imposed.  ``perturb``:
    relative std of i.i.d. noise added to the loss tail's inputs (the disparities and poses the
    networks hand to train_loss), value substituted with the graph kept."""
    x = g["x"]
    N, L, C, H, W = x.shape
    K, invK = D.intrinsics(W, H)
    bins = g.get("bins")
    emb = 21 if bins is not None else 0
    nb = bins.shape[1] if bins is not None else 1
    spec = O.param_spec(arch, C, tuple(levels), embedding_levels=emb)
    scales = tuple(DEFAULT_SCALES[l] for l in levels)
    f = g["flat"].to(dt).clone().requires_grad_(True)
    P = O.unflatten(f, spec)
    with O.forced_decisions(g["decisions"]):
        d_o, p_o = O.model_forward(P, x.to(dt), source_ids, target_id, arch=arch,
                                   scale_levels=tuple(levels),
                                   mpi_bins=None if bins is None else bins.to(dt), embedding_levels=emb)
    if perturb:
        gen = torch.Generator().manual_seed(seed)
        noise = lambda t: t + (t * perturb * torch.randn(t.shape, generator=gen, dtype=t.dtype)).detach()
        d_o = [noise(d) for d in d_o]
        p_o = [(noise(r), noise(t)) for r, t in p_o]
    cache_o = O.TrainCache(K=K.to(dt), invK=invK.to(dt), target_id=target_id,
                           source_ids=tuple(source_ids), scales=scales)
    am = g["automasking"]
    # MPI: the planes are the loss batch, each with its sample's frames and poses (O.mpi_train_loss)
    xt = x.to(dt).repeat_interleave(nb, 0) if nb > 1 else x.to(dt)
    pt = [(r.repeat_interleave(nb, 0), t.repeat_interleave(nb, 0)) for r, t in p_o] if nb > 1 else p_o
    par_o = O.Params(target_size=(W, H), batch_size=N * nb, automasking=am)
    forced = [s.unsqueeze(1).long() + (1 if am else 0) for s in g["sel"]]
    auto_o = O.automasking_loss(xt, xt[:, target_id - 1], source_ids) if am else None
    lo = O.loss_from_outputs(d_o, pt, xt, auto_o, cache_o, par_o, forced_sel=forced,
                             forced_cells=g["cells"])
    lo.backward()
    fwd = ([d.detach().double() for d in d_o], torch.cat([torch.cat([r, t], 1) for r, t in p_o], 0).detach().double())
    return f.grad.double(), fwd, lo.item(), spec


def oracle_bounds(g, o=None, eps=2.0 ** -23, arch=18, levels=(2, 3, 4, 5), target_id=2,
                  source_ids=(1, 3)):
    """Two references for judging the GPU gradient, both from the oracle with every GPU decision
    imposed:
      floor[k]  per-tensor error of the SAME oracle run in fp32 vs fp64 (the fp32 noise floor),
                plus the forward outputs' floors under "__disp<s>", "__pose", "__loss";
      sens[k]   per-tensor relative change of the fp64 gradient when the loss tail's inputs (the
                disparities and poses the networks hand to train_loss) carry relative noise of
                one fp32 ulp (``eps``): how far an fp32-accurate forward can legitimately move
                that gradient.  Large for cancelling sums -- e.g. a decoder head's bias gradient,
                a sum of ~1e6 full-resolution pixel gradients of both signs.
    ``o``: the fp64 result of ``run`` (its gradient is the unperturbed base); recomputed if None."""
    kw = dict(arch=arch, levels=levels, target_id=target_id, source_ids=source_ids)
    if o is None:
        g64, f64, l64, spec = _oracle_grad(g, torch.float64, **kw)
    else:
        g64, f64, l64 = o["grad"].double(), (o["disps"], o["pose"]), o["loss"]
        spec = O.param_spec(arch, g["x"].shape[2], tuple(levels),
                            embedding_levels=21 if g.get("bins") is not None else 0)
    g32, f32, l32, _ = _oracle_grad(g, torch.float32, **kw)
    floor = per_tensor(spec, g32, g64)
    for s_, (a, b) in enumerate(zip(f32[0], f64[0])):
        floor[f"__disp{s_}"] = D.rel_err(a, b)
    floor["__pose"] = D.rel_err(f32[1], f64[1])
    floor["__loss"] = abs(l32 - l64) / abs(l64)
    pert, _, _, _ = _oracle_grad(g, torch.float64, perturb=eps, seed=1, **kw)
    sens = per_tensor(spec, pert, g64)
    return floor, sens


def grad_bounds(floor, sens, abs_floor=2e-5):
    """Per-tensor gradient bound: 4x the oracle's own fp32 floor, 4x its 1-ulp forward
    sensitivity, and an absolute floor for the accumulation-order noise of well-conditioned
    tensors (the GPU sums in other orders than torch-CPU)."""
    return {k: max(4 * floor[k], 4 * sens[k], abs_floor) for k in sens}


def check_step(g, o, errs, floor, sens, label=""):
    """The full-step assertions shared by the model parity tests: loss, forward outputs, and every
    gradient tensor within its bound (grad_bounds).  Prints the tightest margins."""
    assert abs(g["loss"] - o["loss"]) <= max(1e-6, 4 * floor["__loss"]) * abs(o["loss"]), \
        (g["loss"], o["loss"], floor["__loss"])
    for s_, (a, b) in enumerate(zip(g["disps"], o["disps"])):
        assert D.rel_err(a, b) < max(1e-5, 4 * floor[f"__disp{s_}"]), s_
    assert D.rel_err(g["pose"], o["pose"]) < max(1e-5, 4 * floor["__pose"])
    bound = grad_bounds(floor, sens)
    ratio = sorted(((errs[k] / bound[k], k) for k in bound), reverse=True)
    print(f"\n{label} loss {g['loss']:.7f} vs {o['loss']:.7f}; tightest err/bound: " +
          ", ".join(f"{k} {errs[k]:.2e}/{bound[k]:.2e} (floor {floor[k]:.1e}, sens {sens[k]:.1e})"
                    for _, k in ratio[:4]))
    bad = {k: (errs[k], bound[k]) for k in bound if errs[k] > bound[k]}
    assert not bad, bad
    return max(errs.values())
