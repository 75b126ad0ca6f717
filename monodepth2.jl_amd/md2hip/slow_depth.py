"""Config 1 of the measurement plan: ``slow_depth`` (src/simple_depth.jl:1-43), the free-variable
optimisation of one disparity map and two poses against a single triplet.

Per iteration (src/simple_depth.jl:22-42): ``gradient(θ)`` of
``mean(prediction_loss(ssim, warp(disp, x, Ps, ...), target_x)) + smooth_loss(disp, target_x)``
-- one scale at full resolution, no 1e-3 smoothness weight, no mean normalisation of the
disparity, no sigmoid (``disp`` is the parameter itself) -- then ``update!(ADAM(3e-4), θ, ∇)``.
The reference calls a ``warp`` it never defines (defect D1); it is taken to be the
per-scale warp body of ``train_loss`` (src/training.jl:48-57), as in the oracle.

The whole loss and its pullback are one ``md2_loss_fwd_bwd`` call (the fused photometric +
smoothness kernels); θ = [disp | poses] is one flat device vector updated by ``md2_adam``.
Visualisation / PNG logging of the reference loop (``save_disparity``) is not reproduced.
"""
from __future__ import annotations

from typing import Sequence

from ._lib import check, lib, ptr, stream_of
from .loss import Params, TrainCache, loss_tail


def adam_update(p, g, m, v, step: int, lr: float, beta=(0.9, 0.999), eps=1e-8,
                grad_scale: float = 1.0):
    """``Flux.Optimise.update!(ADAM(lr, beta), p, g)`` on flat fp32 CUDA tensors (in place);
    ``step`` >= 1 counts the updates already applied to this vector plus one."""
    check(lib().md2_adam(ptr(p), ptr(g), ptr(m), ptr(v), p.numel(), lr, beta[0], beta[1], eps,
                         step, grad_scale, stream_of(p.device)), "md2_adam")


class SlowDepth:
    """State of the ``slow_depth`` loop for a batch of N triplets x [N, L, C, H, W] (the reference
    runs N = 1).  ``disp`` [N,1,H,W] and ``poses`` [(rvec [N,3], tvec [N,3])] x 2 are views into
    the flat parameter vector ``theta``."""

    def __init__(self, x, K, invK, *, target_id: int = 2, source_ids: Sequence[int] = (1, 3),
                 min_depth: float = 0.1, max_depth: float = 100.0, lr: float = 3e-4):
        import torch
        if not (x.is_cuda and x.dtype == torch.float32 and x.dim() == 5):
            raise ValueError("x must be a float32 CUDA tensor [N, L, C, H, W]")
        self.x = x.contiguous()
        N, L, Cc, H, W = x.shape
        self.N, self.H, self.W = N, H, W
        self.cache = TrainCache(K=K, invK=invK, scales=(1.0,), target_id=target_id,
                                source_ids=tuple(source_ids))
        self.params = Params(target_size=(W, H), batch_size=N, automasking=False,
                             min_depth=min_depth, max_depth=max_depth)
        self.lr = lr
        nd = N * H * W
        dev = x.device
        self.theta = torch.zeros(nd + 2 * N * 6, dtype=torch.float32, device=dev)
        self.grad = torch.zeros_like(self.theta)
        self.m = torch.zeros_like(self.theta)
        self.v = torch.zeros_like(self.theta)
        self.disp = self.theta[:nd].view(N, 1, H, W)
        self.pose_rows = self.theta[nd:].view(2 * N, 6)      # row s*N+i = (rvec, tvec)
        # src/simple_depth.jl:8-13: disp = 0.5; rvec = [0, 0, 0.01], tvec = 0 per source
        self.disp.fill_(0.5)
        self.pose_rows[:, 2] = 0.01
        self.t = 0

    @property
    def poses(self):
        N = self.N
        return [(self.pose_rows[s * N:(s + 1) * N, :3], self.pose_rows[s * N:(s + 1) * N, 3:])
                for s in range(2)]

    def evaluate(self, visualize: bool = False):
        """The loss and its gradient at the current θ (the ``gradient(θ) do ... end`` body)."""
        return loss_tail([self.disp], self.poses, self.x, None, self.cache, self.params,
                         smooth_weights=[1.0], divisor=1.0, smooth_normalize=False,
                         sigmoid_grad=False, visualize=visualize)

    def step(self):
        """One iteration: gradient, then ADAM on θ.  Returns the loss (device tensor [1])."""
        r = self.evaluate()
        nd = self.N * self.H * self.W
        self.grad[:nd].copy_(r["d_disp"][0].reshape(-1))
        self.grad[nd:].copy_(r["d_pose"].reshape(-1))
        self.t += 1
        adam_update(self.theta, self.grad, self.m, self.v, self.t, self.lr)
        return r["loss"]


def slow_depth(x, K, invK, *, iters: int = 500, lr: float = 3e-4, target_id: int = 2,
               source_ids: Sequence[int] = (1, 3), min_depth: float = 0.1,
               max_depth: float = 100.0, log_step: int = 0, callback=None):
    """Run the loop; returns (disp [N,1,H,W], poses, losses [iters] on the host).
    ``callback(iter, state)`` is called every ``log_step`` iterations and at iteration 1 (the
    reference's logging cadence, src/simple_depth.jl:23,44-60)."""
    import torch
    st = SlowDepth(x, K, invK, target_id=target_id, source_ids=source_ids, min_depth=min_depth,
                   max_depth=max_depth, lr=lr)
    losses = torch.empty(iters, dtype=torch.float32, device=x.device)
    for it in range(1, iters + 1):
        losses[it - 1:it].copy_(st.step())
        if callback is not None and log_step and (it % log_step == 0 or it == 1):
            callback(it, st)
    return st.disp, st.poses, losses.cpu()
