# MD2HIP.jl -- the Julia host binding of libmd2hip.so (include/md2.h) for Monodepth2.jl.
#
# Drop-in for the reference's GPU hot path: `include("MD2HIP.jl")` from src/Monodepth.jl (after
# `using AMDGPU, ChainRulesCore`), then use MD2HIP.HIPModel / MD2HIP.train_loss where the reference
# uses Model / train_loss (src/training.jl:21-78, scripts/script.jl:84-86).  Every op below is a
# forward `ccall` plus a `ChainRulesCore.rrule` whose pullback is the library's hand-written HIP
# pullback -- the reference's own plugin mechanism (src/utils.jl:134-145, src/repeat.jl:44-69).
#
# Julia is not installed in the build container: this file is the binding a maintainer adds; the
# Python mirror monodepth2.jl_amd/md2hip/ makes the same calls and is what the tests execute.
#
# Layout contract (INTEGRATION.md): Julia column-major (W,H,C,N) arrays have the bytes of the
# library's C-order [n][c][h][w]; 3x3 matrices go row-major (`vec(permutedims(K))`); Flux Conv
# weights (kw,kh,cin,cout) are true convolutions -> flipped once into the library's
# cross-correlation layout by `flat_params`.
module MD2HIP

using AMDGPU
using ChainRulesCore
import Flux

const lib = get(ENV, "MD2HIP_LIB",
                joinpath(@__DIR__, "..", "monodepth2.jl_amd", "lib", "libmd2hip.so"))

const ABI_VERSION = 2                                  # include/md2.h MD2_ABI_VERSION
function __init__()
    v = ccall((:md2_abi_version, lib), Cint, ())
    v == ABI_VERSION || error("libmd2hip at ", lib, " has ABI version ", v,
                              ", MD2HIP.jl expects ", ABI_VERSION, ": rebuild or update the binding")
end

check(rc) = rc == 0 || error("libmd2hip (", rc, "): ",
                             unsafe_string(ccall((:md2_last_error, lib), Cstring, ())))
stream_ptr() = AMDGPU.stream().stream                  # hipStream_t of the task-local stream
rowmajor(M) = ntuple(i -> Float32(M[(i - 1) ÷ 3 + 1, (i - 1) % 3 + 1]), 9)
pad5(v, T) = ntuple(i -> i <= length(v) ? T(v[i]) : zero(T), 5)
ptr(a) = a === nothing ? C_NULL : pointer(a)

# ------------------------------------------------------------------------------------------------
# C structs (field order and types exactly as include/md2.h)
# ------------------------------------------------------------------------------------------------
struct ModelCfg                                        # md2_model_cfg
    arch::Cint; in_channels::Cint; batch::Cint; width::Cint; height::Cint
    n_levels::Cint; scale_levels::NTuple{5,Cint}
    K::NTuple{9,Cfloat}; invK::NTuple{9,Cfloat}
    min_depth::Cfloat; max_depth::Cfloat; disparity_smoothness::Cfloat
    scales::NTuple{5,Cfloat}; automasking::Cint
    target::Cint; src0::Cint; src1::Cint
    embedding_levels::Cint; num_bins::Cint
end

# Params / TrainCache of src/Monodepth.jl:37-60 -> md2_model_cfg.  MPI mode (src/model.jl:1-55):
# embedding_levels = 21 (DepthDecoder(; embedding_levels)) and num_bins disparity planes, batch 1
function ModelCfg(arch, in_ch, scale_levels, p, c; embedding_levels=0, num_bins=1)
    ModelCfg(arch, in_ch, p.batch_size, p.target_size..., length(scale_levels),
             pad5(scale_levels, Cint), rowmajor(c.K), rowmajor(c.invK),
             p.min_depth, p.max_depth, p.disparity_smoothness, pad5(c.scales, Cfloat),
             p.automasking, c.target_id - 1, c.source_ids[1] - 1, c.source_ids[2] - 1,
             embedding_levels, num_bins)
end

struct LossCfg                                         # md2_loss_cfg
    n::Cint; c::Cint; width::Cint; height::Cint; nscales::Cint
    scale_w::NTuple{5,Cint}; scale_h::NTuple{5,Cint}
    smooth_weight::NTuple{5,Cfloat}; divisor::Cfloat; smooth_normalize::Cint
    K::NTuple{9,Cfloat}; invK::NTuple{9,Cfloat}
    min_depth::Cfloat; max_depth::Cfloat
    x_sample_stride::Clonglong; x_frame_stride::Clonglong
    target::Cint; src0::Cint; src1::Cint; invert_mask::Cint; sigmoid_grad::Cint
end

struct LossOut                                         # md2_loss_out
    loss::Ptr{Float32}; terms::Ptr{Float32}
    d_disp::NTuple{5,Ptr{Float32}}; d_pose::Ptr{Float32}
    vis_loss::Ptr{Float32}; vis_sel::Ptr{Int8}; vis_warped::Ptr{Float32}
    vis_cell::Ptr{Int32}                               # parity diagnostics (not used here)
end

struct WarpCfg                                         # md2_warp_cfg
    n::Cint; c::Cint; width::Cint; height::Cint; dw::Cint; dh::Cint
    K::NTuple{9,Cfloat}; invK::NTuple{9,Cfloat}
    min_depth::Cfloat; max_depth::Cfloat
    x_sample_stride::Clonglong; x_frame_stride::Clonglong
    target::Cint; src0::Cint; src1::Cint
end

struct ConvDesc                                        # md2_conv_desc
    n::Cint; cin::Cint; h::Cint; w::Cint; cout::Cint; kh::Cint; kw::Cint
    stride::Cint; pad::Cint; reflect::Cint; act::Cint
end

# ------------------------------------------------------------------------------------------------
# The model: Model(ResidualNetwork, DepthDecoder, PoseDecoder) with its parameters in ONE flat
# device vector (Flux `params(model)` order, md2_arch_param_info) -- src/model.jl:24-70
# ------------------------------------------------------------------------------------------------
mutable struct HIPModel
    handle::Ptr{Cvoid}
    cfg::ModelCfg
    θ::ROCVector{Float32}          # the trainable parameters, library layout (conv taps as
                                   # cross-correlation); Flux.params(m) == Params([m.θ])
    ∇θ::ROCVector{Float32}         # the library's gradient buffer (same layout)
    m::ROCVector{Float32}; v::ROCVector{Float32}; step::Int   # library ADAM state (update!)
    packed::Bool                   # the library's packed conv weights reflect θ
end

# Flux.params(model) / gradient(θ) / Flux.Optimise.update!(opt, θ, ∇) (scripts/script.jl:84-86):
# the one trainable array is θ.  ADAM is elementwise, so training θ in the library layout is the
# same arithmetic as training the Flux layout; get_params / set_params! convert for checkpoints.
Flux.@functor HIPModel (θ,)
Flux.trainable(m::HIPModel) = (θ = m.θ,)

function param_count(cfg::ModelCfg)
    ne, nel = Ref{Clonglong}(), Ref{Clonglong}()
    check(ccall((:md2_arch_param_count, lib), Cint, (Ref{ModelCfg}, Ref{Clonglong}, Ref{Clonglong}),
                cfg, ne, nel))
    return Int(ne[]), Int(nel[])
end

# (name, shape, 0-based offset) of table entry i (0-based)
function param_info(cfg::ModelCfg, i)
    name = Vector{UInt8}(undef, 128); nd = Ref{Cint}(); shape = zeros(Cint, 4); off = Ref{Clonglong}()
    check(ccall((:md2_arch_param_info, lib), Cint,
                (Ref{ModelCfg}, Cint, Ptr{UInt8}, Cint, Ref{Cint}, Ptr{Cint}, Ref{Clonglong}),
                cfg, i, name, length(name), nd, shape, off))
    return unsafe_string(pointer(name)), Tuple(Int.(shape[1:nd[]])), Int(off[])
end

# Flux params -> the library's flat vector: conv weights (kw,kh,cin,cout) flipped in both spatial
# axes (true convolution -> cross-correlation); everything else copied as is.  `ps` iterates in
# Flux `params(model)` order, which is the table order.
function flat_params(cfg::ModelCfg, ps)
    ne, nel = param_count(cfg)
    flat = Vector{Float32}(undef, nel)
    for (i, p) in enumerate(ps)
        name, shape, off = param_info(cfg, i - 1)
        length(p) == prod(shape) || error("parameter $name: Flux size $(size(p)) vs table $shape")
        a = Array{Float32}(p)
        ndims(a) == 4 && (a = a[end:-1:1, end:-1:1, :, :])
        flat[off+1:off+length(a)] = vec(a)
    end
    ne == length(collect(ps)) || error("Flux model has a different parameter count than the table")
    return ROCVector{Float32}(flat)
end

function HIPModel(cfg::ModelCfg, θ::ROCVector{Float32})
    ∇θ = similar(θ); h = Ref{Ptr{Cvoid}}()
    check(ccall((:md2_model_create, lib), Cint,
                (Ref{ModelCfg}, Ptr{Float32}, Ptr{Float32}, Ref{Ptr{Cvoid}}), cfg, θ, ∇θ, h))
    m = HIPModel(h[], cfg, θ, ∇θ, fill!(similar(θ), 0), fill!(similar(θ), 0), 0, false)
    repack!(m)
    finalizer(x -> ccall((:md2_model_destroy, lib), Cint, (Ptr{Cvoid},), x.handle), m)
end

# after the caller changed m.θ in place (Flux.Optimise.update!, loading a checkpoint): re-pack the
# library's conv weights.  train_loss does it by itself after every pullback (see below).
function repack!(m::HIPModel)
    check(ccall((:md2_model_repack, lib), Cint, (Ptr{Cvoid}, Ptr{Cvoid}), m.handle, stream_ptr()))
    m.packed = true
    return m
end

# (m)(x, source_ids, target_id) -- disparities (Julia (w,h,1,n) views of library memory) and
# poses of the last forward (src/model.jl:24-55)
function outputs(m::HIPModel)
    d = Vector{Ptr{Float32}}(undef, 5); w = zeros(Cint, 5); h = zeros(Cint, 5); pose = Ref{Ptr{Float32}}()
    check(ccall((:md2_model_outputs, lib), Cint,
                (Ptr{Cvoid}, Ptr{Ptr{Float32}}, Ptr{Cint}, Ptr{Cint}, Ref{Ptr{Float32}}),
                m.handle, d, w, h, pose))
    n = m.cfg.batch
    np = m.cfg.embedding_levels > 0 ? Int(m.cfg.num_bins) : 1          # MPI: plane images
    disps = [unsafe_wrap(ROCArray, d[k], (Int(w[k]), Int(h[k]), 1, n * np)) for k in 1:m.cfg.n_levels]
    return disps, unsafe_wrap(ROCArray, pose[], (6, 2n))
end

"""
    HIPModel(model, cache, params; num_bins=32)

The HIP model of a reference `Model(encoder, depth_decoder, pose_decoder)` (src/model.jl:24-29,
built as in scripts/script.jl:77-81) for one `TrainCache` / `Params`: the architecture (ResNet
depth, input channels, `scale_levels`, `embedding_levels`) is read off the Flux model and its
parameters are copied (conv kernels flipped into the library layout) into the flat θ.
"""
function HIPModel(model, cache, params; num_bins=32)
    enc, dec = model.encoder, model.depth_decoder
    ch = collect(enc.stages)
    levels = cumsum([length(b) for b in dec.branches])
    emb = size(dec.branches[1][1].c1.d.weight, 3) - ch[end]
    ps = collect(Flux.params(model))
    in_ch = size(ps[1], 3)                         # the stem conv (kw,kh,cin,64)
    for arch in (ch[end] == 2048 ? (50,) : (18, 34))
        cfg = ModelCfg(arch, in_ch, levels, params, cache; embedding_levels=emb,
                       num_bins=emb > 0 ? num_bins : 1)
        param_count(cfg)[1] == length(ps) || continue
        return HIPModel(cfg, flat_params(cfg, ps))
    end
    error("HIPModel: the Flux model matches no ResidualNetwork(18/34/50) + DepthDecoder + PoseDecoder table")
end

"""
    (m::HIPModel)(x, source_ids, target_id) -> (disparities, poses)

`(m::Model)(x, source_ids, target_id)` of src/model.jl:31-55 (called by train_loss at
src/training.jl:26 and bare at scripts/script.jl:93) on the HIP path, forward only: `disparities`
one (w,h,1,n) array per scale level ((w,h,1,n*num_bins) in MPI mode), `poses` one
`(rvec = (3,n), tvec = (3,1,n))` per source (the fields train_loss reads of `Pose`).  The rrule's
pullback runs the library's backward from the caller's cotangents (md2_model_backward_from), so
the reference's own train_loss can be differentiated through it by Zygote.  `source_ids` /
`target_id` must be the ones the model was built with.
"""
function (m::HIPModel)(x::ROCArray{Float32,5}, source_ids, target_id)
    (target_id - 1, source_ids[1] - 1, source_ids[2] - 1) == (m.cfg.target, m.cfg.src0, m.cfg.src1) ||
        error("HIPModel: target_id / source_ids differ from the config the model was built with")
    _forward(m, m.θ, x)
end

function _forward(m::HIPModel, θ::ROCVector{Float32}, x::ROCArray{Float32,5})
    θ === m.θ || error("HIPModel: θ must be the model's own parameter vector")
    m.packed || repack!(m)
    check(ccall((:md2_model_forward, lib), Cint,
                (Ptr{Cvoid}, Ptr{Float32}, Ptr{Ptr{Float32}}, Ptr{Ptr{Float32}}, Ptr{Cvoid}),
                m.handle, x, C_NULL, C_NULL, stream_ptr()))
    disps, pose = outputs(m)
    n = m.cfg.batch
    poses = [(rvec = pose[1:3, (s - 1) * n + 1:s * n], tvec = reshape(pose[4:6, (s - 1) * n + 1:s * n], 3, 1, n))
             for s in 1:2]
    return [copy(d) for d in disps], poses        # copies: the next forward reuses the buffers
end

function ChainRulesCore.rrule(::typeof(_forward), m::HIPModel, θ::ROCVector{Float32}, x)
    y = _forward(m, θ, x)
    function forward_pullback(Δ)
        Δd, Δp = unthunk(Δ[1]), unthunk(Δ[2])
        keep = Any[]
        dptrs = fill(Ptr{Float32}(C_NULL), 5)
        if !(Δd isa AbstractZero)
            for (k, d) in enumerate(Δd)
                d = unthunk(d)
                d isa AbstractZero && continue
                a = ROCArray{Float32}(d); push!(keep, a); dptrs[k] = pointer(a)
            end
        end
        dpose = Ptr{Float32}(C_NULL)
        if !(Δp isa AbstractZero)
            n = m.cfg.batch; P = fill!(ROCArray{Float32}(undef, 6, 2n), 0f0)
            for (s, p) in enumerate(Δp)
                p = unthunk(p)
                p isa AbstractZero && continue
                r, t = unthunk(p.rvec), unthunk(p.tvec)
                r isa AbstractZero || (P[1:3, (s - 1) * n + 1:s * n] .= reshape(r, 3, n))
                t isa AbstractZero || (P[4:6, (s - 1) * n + 1:s * n] .= reshape(t, 3, n))
            end
            push!(keep, P); dpose = pointer(P)
        end
        check(ccall((:md2_model_backward_from, lib), Cint,
                    (Ptr{Cvoid}, Ptr{Ptr{Float32}}, Ptr{Float32}, Ptr{Cvoid}),
                    m.handle, dptrs, dpose, stream_ptr()))
        AMDGPU.synchronize()                 # the cotangent copies in `keep` are read asynchronously
        m.packed = false
        return NoTangent(), NoTangent(), copy(m.∇θ), NoTangent()
    end
    return y, forward_pullback
end

# the loss-tail config of this model (for the visualisation pass)
function loss_cfg(m::HIPModel)
    c = m.cfg; disps, _ = outputs(m)
    LossCfg(c.batch, c.in_channels, c.width, c.height, c.n_levels,
            pad5([size(d, 1) for d in disps], Cint), pad5([size(d, 2) for d in disps], Cint),
            pad5([c.disparity_smoothness * s for s in c.scales[1:c.n_levels]], Cfloat),
            Float32(c.n_levels), 1, c.K, c.invK, c.min_depth, c.max_depth,
            3 * c.in_channels * c.height * c.width, c.in_channels * c.height * c.width,
            c.target, c.src0, c.src1, (c.src0 < c.target ? 1 : 0) | (c.src1 < c.target ? 2 : 0), 1)
end

"""
    train_loss(m, x, auto_loss, cache, params, do_visualization=false)

`train_loss` of src/training.jl:21-78 on the HIP path, with the reference's return convention:
`(loss, vis_disparity, vis_warped, vis_loss)` where `loss` is a host `Float32` scalar
(`loss / T(length(cache.scales))`, :77) and the visualisation outputs are host arrays
(`cpu(disparities[end])` (W,H,1,n), `cpu.(warped_images)` two (W,H,C,n), `cpu(warp_loss)`
(W,H,1,n); `nothing`s when `do_visualization` is false, :34-37,71-74).  The forward also runs the
fused loss-tail pullback; the rrule finishes the backward.  `cache` / `params` are the ones the
model was built with (md2_model_cfg): any field that differs raises (`check_config`).

Zygote: `gradient(() -> train_loss(m, x, ...)[1], Flux.params(m))` (the implicit-parameter loop
of scripts/script.jl:84-86, src/simple_depth.jl:25-42) returns the gradient under `m.θ`, in
m.θ's own layout, so `Flux.Optimise.update!(opt, Flux.params(m), ∇)` updates m.θ consistently.
"""
function train_loss(m::HIPModel, x::ROCArray{Float32,5}, auto_loss, cache, params,
                    do_visualization::Bool=false)
    check_config(m, cache, params)
    _train_loss(m, m.θ, x, auto_loss, do_visualization)     # m.θ read in traced code: accum_param
end

# The executor's kernels, buffers and loss-tail weights are built for ONE (Params, TrainCache)
# (md2_model_cfg).  The reference reads them per call (src/training.jl:40-67), so a caller passing
# a different cache / params must get an error, not the build-time config's loss.
function check_config(m::HIPModel, cache, params)
    c = m.cfg
    bad = String[]
    (params.batch_size, params.target_size...) == (c.batch, c.width, c.height) ||
        push!(bad, "batch_size / target_size")
    Float32(params.min_depth) == c.min_depth && Float32(params.max_depth) == c.max_depth ||
        push!(bad, "min_depth / max_depth")
    Float32(params.disparity_smoothness) == c.disparity_smoothness || push!(bad, "disparity_smoothness")
    Cint(params.automasking) == c.automasking || push!(bad, "automasking")
    (cache.target_id - 1, cache.source_ids[1] - 1, cache.source_ids[2] - 1) == (c.target, c.src0, c.src1) ||
        push!(bad, "target_id / source_ids")
    Float32.(cache.scales) == collect(c.scales[1:c.n_levels]) || push!(bad, "scales")
    rowmajor(cache.K) == c.K && rowmajor(cache.invK) == c.invK || push!(bad, "K / invK")
    isempty(bad) || error("train_loss: ", join(bad, ", "), " differ from the config the HIPModel was ",
                          "built with (md2_model_cfg); build a HIPModel for this cache / params")
    return nothing
end

function _train_loss(m::HIPModel, θ::ROCVector{Float32}, x::ROCArray{Float32,5}, auto_loss,
                     do_visualization::Bool)
    θ === m.θ || error("train_loss: θ must be the model's own parameter vector")
    m.packed || repack!(m)               # θ may have been updated in place since the last step
    loss = ROCVector{Float32}(undef, 1)
    check(ccall((:md2_model_forward_loss, lib), Cint,
                (Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                m.handle, x, ptr(auto_loss), loss, C_NULL, stream_ptr()))
    l = Array(loss)[1]                   # host scalar, as the reference's mean(...) / T(...)
    do_visualization || return (l, nothing, nothing, nothing)
    disps, pose = outputs(m)
    cfg = loss_cfg(m); n = m.cfg.batch; c = m.cfg.in_channels; W = m.cfg.width; H = m.cfg.height
    vis_loss = ROCArray{Float32}(undef, W, H, n, cfg.nscales)
    vis_sel = ROCArray{Int8}(undef, W, H, n, cfg.nscales)
    vis_warped = ROCArray{Float32}(undef, W, H, c, n, 2)
    tmp = ROCVector{Float32}(undef, 1)
    ws = ROCVector{UInt8}(undef, ccall((:md2_loss_workspace_size, lib), Csize_t, (Ref{LossCfg},), cfg))
    out = LossOut(pointer(tmp), C_NULL, ntuple(_ -> Ptr{Float32}(C_NULL), 5), C_NULL,
                  pointer(vis_loss), pointer(vis_sel), pointer(vis_warped), C_NULL)
    dptrs = [pointer(d) for d in disps]
    check(ccall((:md2_loss_fwd_bwd, lib), Cint,
                (Ref{LossCfg}, Ptr{Ptr{Float32}}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Cfloat,
                 Ref{LossOut}, Ptr{UInt8}, Ptr{Cvoid}),
                cfg, dptrs, pose, x, ptr(auto_loss), 1f0, out, ws, stream_ptr()))
    # training.jl:34-37,71-74: last disparity, both warped sources and the last scale's loss map
    return (l, Array(disps[end]), (Array(vis_warped[:, :, :, :, 1]), Array(vis_warped[:, :, :, :, 2])),
            Array(reshape(vis_loss[:, :, :, end], W, H, 1, n)))
end

# gradient(θ) do train_loss(...)[1] end: the remaining backward segments -> m.∇θ.  `bucket(off,
# len)` runs after each segment (that flat range is final) so a DP caller can all-reduce it.
function gradient!(m::HIPModel; bucket=(off, len) -> nothing)
    nseg = ccall((:md2_model_num_segments, lib), Cint, (Ptr{Cvoid},), m.handle)
    off, len = Ref{Clonglong}(), Ref{Clonglong}()
    for k in 0:nseg-1
        check(ccall((:md2_model_backward_segment, lib), Cint,
                    (Ptr{Cvoid}, Cint, Ref{Clonglong}, Ref{Clonglong}, Ptr{Cvoid}),
                    m.handle, k, off, len, stream_ptr()))
        bucket(off[], len[])
    end
    return m.∇θ
end

# Zygote: d(train_loss(...)[1])/dθ.  The loss cotangent enters the library's backward itself
# (md2_model_loss_cotangent scales the fused loss tail's d disp / d pose before segment 0).  The
# θ tangent is a fresh array in θ's own (library) layout -- what Flux.Optimise.update! adds to
# θ; the Flux-layout gradient (true-convolution kernels) is flux_gradient(m).  The caller is
# expected to update θ next, so the packed weights are marked stale (re-packed by the next
# train_loss, or already by the library's own update!).
function ChainRulesCore.rrule(::typeof(_train_loss), m::HIPModel, θ::ROCVector{Float32}, x, auto_loss,
                              do_visualization::Bool)
    y = _train_loss(m, θ, x, auto_loss, do_visualization)
    function train_loss_pullback(Δ)
        Δl = unthunk(Δ[1])
        Δl = Δl isa AbstractZero ? 0f0 : Float32(Δl)
        check(ccall((:md2_model_loss_cotangent, lib), Cint, (Ptr{Cvoid}, Cfloat, Ptr{Cvoid}),
                    m.handle, Δl, stream_ptr()))
        gradient!(m)
        m.packed = false
        return (NoTangent(), NoTangent(), copy(m.∇θ), NoTangent(), NoTangent(), NoTangent())
    end
    return y, train_loss_pullback
end

# the last gradient in Flux layout (Flux.params order, conv kernels as true convolutions): what
# Zygote returns for a Flux Model's params -- for comparing against / exporting to the reference
function flux_gradient(m::HIPModel)
    ∇flux = similar(m.∇θ)
    check(ccall((:md2_model_get_grads, lib), Cint, (Ptr{Cvoid}, Ptr{Float32}, Ptr{Cvoid}),
                m.handle, ∇flux, stream_ptr()))
    return ∇flux
end

# Flux-layout parameters in / out of the model (device copies with the conv taps flipped)
function set_params!(m::HIPModel, flux::ROCVector{Float32})
    check(ccall((:md2_model_set_params, lib), Cint, (Ptr{Cvoid}, Ptr{Float32}, Ptr{Cvoid}),
                m.handle, flux, stream_ptr()))
    m.packed = true                      # md2_model_set_params re-packs
    return m
end
function get_params(m::HIPModel)
    flux = similar(m.θ)
    check(ccall((:md2_model_get_params, lib), Cint, (Ptr{Cvoid}, Ptr{Float32}, Ptr{Cvoid}),
                m.handle, flux, stream_ptr()))
    return flux
end

# update!(ADAM(η), θ, ∇θ) -- Flux ADAM, β = (0.9, 0.999), ε = 1e-8 (scripts/script.jl:85)
function update!(m::HIPModel, η; β=(0.9f0, 0.999f0), ϵ=1f-8, grad_scale=1f0)
    m.step += 1
    check(ccall((:md2_model_adam, lib), Cint,
                (Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}, Cfloat, Cfloat, Cfloat, Cfloat, Cint, Cfloat, Ptr{Cvoid}),
                m.handle, m.m, m.v, η, β[1], β[2], ϵ, m.step, grad_scale, stream_ptr()))
    m.packed = true                      # md2_model_adam re-packs
    return m
end

# eval_disparity(m, x) -- src/model.jl:63; x::(W,H,C,n), n <= batch
function eval_disparity(m::HIPModel, x::ROCArray{Float32,4})
    d = Vector{Ptr{Float32}}(undef, 5)
    check(ccall((:md2_model_eval_disparity, lib), Cint,
                (Ptr{Cvoid}, Ptr{Float32}, Cint, Ptr{Ptr{Float32}}, Ptr{Cvoid}),
                m.handle, x, size(x, 4), d, stream_ptr()))
    W, H = m.cfg.width, m.cfg.height; lv = m.cfg.scale_levels
    return [unsafe_wrap(ROCArray, d[k], (W >> (5 - lv[k]), H >> (5 - lv[k]), 1, size(x, 4)))
            for k in 1:m.cfg.n_levels]
end

# ------------------------------------------------------------------------------------------------
# Op-level forward + rrule pairs (src/utils.jl, src/training.jl): for callers that keep Flux for
# the networks and differentiate the loss ops one at a time.
# ------------------------------------------------------------------------------------------------
struct SSIM end                                        # src/utils.jl:17-43 (constants built in)

function (s::SSIM)(x::ROCArray{Float32,4}, y::ROCArray{Float32,4})
    W, H, C, N = size(x); out = similar(x)
    check(ccall((:md2_ssim_fwd, lib), Cint,
                (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{Cvoid}),
                x, y, N, C, H, W, out, stream_ptr()))
    return out
end

function ChainRulesCore.rrule(s::SSIM, x::ROCArray{Float32,4}, y::ROCArray{Float32,4})
    out = s(x, y)
    function ssim_pullback(Δ)
        W, H, C, N = size(x); dx = similar(x); dy = similar(y)
        dout = ROCArray{Float32}(unthunk(Δ))
        check(ccall((:md2_ssim_bwd, lib), Cint,
                    (Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32},
                     Ptr{Float32}, Ptr{Cvoid}), x, y, dout, N, C, H, W, dx, dy, stream_ptr()))
        return NoTangent(), dx, dy
    end
    return out, ssim_pullback
end

# Backproject: (b)(depth (1, W*H, N), invK) -> (3, W*H, N)   src/utils.jl:45-69
struct Backproject; width::Int; height::Int; end
function (b::Backproject)(depth::ROCArray{Float32,3}, invK)
    N = size(depth, 3); out = ROCArray{Float32}(undef, 3, b.width * b.height, N)
    iK = collect(rowmajor(invK))
    check(ccall((:md2_backproject_fwd, lib), Cint,
                (Ptr{Float32}, Cint, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                depth, N, b.width, b.height, iK, out, stream_ptr()))
    return out
end
function ChainRulesCore.rrule(b::Backproject, depth::ROCArray{Float32,3}, invK)
    out = b(depth, invK)
    function backproject_pullback(Δ)
        dd = similar(depth); dout = ROCArray{Float32}(unthunk(Δ)); iK = collect(rowmajor(invK))
        check(ccall((:md2_backproject_bwd, lib), Cint,
                    (Ptr{Float32}, Cint, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                    dout, size(depth, 3), b.width, b.height, iK, dd, stream_ptr()))
        return NoTangent(), dd, NoTangent()            # invK: TrainCache constant
    end
    return out, backproject_pullback
end

# Project: (p)(points (3, W*H, N), K, R (3,3,N), t (3,1,N)) -> (2, W, H, N)   src/utils.jl:71-103
struct Project; width::Int; height::Int; end
rowmajor_batch(R) = ROCArray{Float32}(permutedims(Array(R), (2, 1, 3)))   # [n][3][3] row-major
function (p::Project)(points::ROCArray{Float32,3}, K, R, t)
    N = size(points, 3); out = ROCArray{Float32}(undef, 2, p.width, p.height, N)
    check(ccall((:md2_project_fwd, lib), Cint,
                (Ptr{Float32}, Cint, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                points, N, p.width, p.height, collect(rowmajor(K)), rowmajor_batch(R),
                ROCArray{Float32}(t), out, stream_ptr()))
    return out
end
function ChainRulesCore.rrule(p::Project, points::ROCArray{Float32,3}, K, R, t)
    out = p(points, K, R, t)
    function project_pullback(Δ)
        N = size(points, 3); dpts = similar(points)
        dRr = ROCArray{Float32}(undef, 9, N); dt = ROCArray{Float32}(undef, 3, 1, N)
        ws = ROCVector{UInt8}(undef, ccall((:md2_project_workspace_size, lib), Csize_t,
                                           (Cint, Cint, Cint), N, p.width, p.height))
        check(ccall((:md2_project_bwd, lib), Cint,
                    (Ptr{Float32}, Cint, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                     Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{UInt8}, Ptr{Cvoid}),
                    points, N, p.width, p.height, collect(rowmajor(K)), rowmajor_batch(R),
                    ROCArray{Float32}(t), ROCArray{Float32}(unthunk(Δ)), dpts, dRr, dt, ws, stream_ptr()))
        dR = permutedims(reshape(dRr, 3, 3, N), (2, 1, 3))   # back to column-major (3,3,N)
        return NoTangent(), dpts, NoTangent(), dR, dt
    end
    return out, project_pullback
end

# grid_sample(x, grid; padding_mode=:border), align_corners=true -- src/training.jl:56
function grid_sample_border(x::ROCArray{Float32,4}, grid::ROCArray{Float32,4})
    Wi, Hi, C, N = size(x); Wo, Ho = size(grid, 2), size(grid, 3)
    out = ROCArray{Float32}(undef, Wo, Ho, C, N)
    check(ccall((:md2_grid_sample_border_fwd, lib), Cint,
                (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{Cvoid}),
                x, grid, N, C, Hi, Wi, Ho, Wo, out, stream_ptr()))
    return out
end
function ChainRulesCore.rrule(::typeof(grid_sample_border), x::ROCArray{Float32,4}, grid::ROCArray{Float32,4})
    out = grid_sample_border(x, grid)
    function grid_sample_pullback(Δ)
        Wi, Hi, C, N = size(x); Wo, Ho = size(grid, 2), size(grid, 3)
        dgrid = similar(grid); dx = fill!(similar(x), 0)
        check(ccall((:md2_grid_sample_border_bwd, lib), Cint,
                    (Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Cint, Cint,
                     Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                    x, grid, ROCArray{Float32}(unthunk(Δ)), N, C, Hi, Wi, Ho, Wo, dgrid, dx, stream_ptr()))
        return NoTangent(), dx, dgrid
    end
    return out, grid_sample_pullback
end

# smooth_loss(disparity (W,H,N), image (W,H,C,N)) -> scalar   src/utils.jl:163-177
function smooth_loss(disp::ROCArray{Float32}, img::ROCArray{Float32,4})
    W, H, C, N = size(img); loss = ROCVector{Float32}(undef, 1)
    ws = ROCVector{UInt8}(undef, ccall((:md2_smooth_loss_workspace_size, lib), Csize_t, (Cint, Cint, Cint), N, W, H))
    check(ccall((:md2_smooth_loss_fwd, lib), Cint,
                (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{UInt8}, Ptr{Cvoid}),
                disp, img, N, C, H, W, loss, ws, stream_ptr()))
    return Array(loss)[1]
end
function ChainRulesCore.rrule(::typeof(smooth_loss), disp::ROCArray{Float32}, img::ROCArray{Float32,4})
    l = smooth_loss(disp, img)
    function smooth_loss_pullback(Δ)
        W, H, C, N = size(img); dd = similar(disp)
        ws = ROCVector{UInt8}(undef, ccall((:md2_smooth_loss_workspace_size, lib), Csize_t, (Cint, Cint, Cint), N, W, H))
        check(ccall((:md2_smooth_loss_bwd, lib), Cint,
                    (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Cfloat, Ptr{Float32}, Ptr{UInt8}, Ptr{Cvoid}),
                    disp, img, N, C, H, W, Float32(unthunk(Δ)), dd, ws, stream_ptr()))
        return NoTangent(), dd, NoTangent()
    end
    return l, smooth_loss_pullback
end

# One scale of train_loss's loop body (src/training.jl:43-62): upsample -> depth -> Backproject ->
# Project -> grid_sample -> photometric_loss -> min over sources [-> _apply_mask].
# disp (dw,dh,1,N); Rt (12, N, 2) = composeT outputs (R row-major, t); x (W,H,C,3,N).
function warp_photometric(cfg::WarpCfg, disp, Rt, x, automask=nothing)
    loss = ROCArray{Float32}(undef, cfg.width, cfg.height, 1, cfg.n)
    ws = ROCVector{UInt8}(undef, ccall((:md2_warp_photometric_workspace_size, lib), Csize_t, (Ref{WarpCfg},), cfg))
    check(ccall((:md2_warp_photometric_fwd, lib), Cint,
                (Ref{WarpCfg}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                 Ptr{Int8}, Ptr{UInt8}, Ptr{Cvoid}),
                cfg, disp, Rt, x, ptr(automask), loss, C_NULL, ws, stream_ptr()))
    return loss
end
function ChainRulesCore.rrule(::typeof(warp_photometric), cfg::WarpCfg, disp, Rt, x, automask=nothing)
    loss = warp_photometric(cfg, disp, Rt, x, automask)
    function warp_photometric_pullback(Δ)
        dd = similar(disp); dRt = similar(Rt)
        ws = ROCVector{UInt8}(undef, ccall((:md2_warp_photometric_workspace_size, lib), Csize_t, (Ref{WarpCfg},), cfg))
        check(ccall((:md2_warp_photometric_bwd, lib), Cint,
                    (Ref{WarpCfg}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                     Ptr{Float32}, Ptr{Float32}, Ptr{UInt8}, Ptr{Cvoid}),
                    cfg, disp, Rt, x, ptr(automask), ROCArray{Float32}(unthunk(Δ)), dd, dRt, ws, stream_ptr()))
        return NoTangent(), NoTangent(), dd, dRt, NoTangent(), NoTangent()
    end
    return loss, warp_photometric_pullback
end

# composeT(so3_exp_map(rvec), tvec, invert) for the 2n poses (src/utils.jl:106-145,185-192);
# pose (6, 2n) = (rvec, tvec) per (source, sample); bit s of invert_mask: source s < target.
function so3_compose(pose::ROCArray{Float32,2}, invert_mask::Integer)
    n = size(pose, 2) ÷ 2; Rt = ROCArray{Float32}(undef, 12, 2n)
    check(ccall((:md2_so3_compose_fwd, lib), Cint, (Ptr{Float32}, Cint, Cint, Ptr{Float32}, Ptr{Cvoid}),
                pose, n, invert_mask, Rt, stream_ptr()))
    return Rt
end
function ChainRulesCore.rrule(::typeof(so3_compose), pose::ROCArray{Float32,2}, invert_mask::Integer)
    Rt = so3_compose(pose, invert_mask)
    function so3_compose_pullback(Δ)
        dpose = similar(pose)
        check(ccall((:md2_so3_compose_bwd, lib), Cint,
                    (Ptr{Float32}, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                    pose, size(pose, 2) ÷ 2, invert_mask, ROCArray{Float32}(unthunk(Δ)), dpose, stream_ptr()))
        return NoTangent(), dpose, NoTangent()
    end
    return Rt, so3_compose_pullback
end

# find_static(dataset, α) -- src/dtk.jl:51-69: per-triplet mean identity-reprojection loss of a
# batch x (W,H,C,3,n) on the GPU; the dataset keeps the files whose score exceeds α
function static_scores(x::ROCArray{Float32,5}; target_id=2, source_ids=(1, 3))
    W, H, C, L, n = size(x); scores = ROCVector{Float32}(undef, n)
    ws = ROCVector{UInt8}(undef, ccall((:md2_static_scores_workspace_size, lib), Csize_t, (Cint, Cint, Cint), n, H, W))
    check(ccall((:md2_static_scores, lib), Cint,
                (Ptr{Float32}, Cint, Cint, Cint, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{UInt8}, Ptr{Cvoid}),
                x, n, C, H, W, target_id - 1, source_ids[1] - 1, source_ids[2] - 1, scores, ws, stream_ptr()))
    return Array(scores)
end

function find_static(dataset, α; batch=16)
    keep = String[]
    for b0 in 1:batch:length(dataset)
        idx = b0:min(length(dataset), b0 + batch - 1)
        x = ROCArray(cat([dataset[i] for i in idx]...; dims=5))
        s = static_scores(x; target_id=dataset.target_id, source_ids=dataset.source_ids)
        append!(keep, dataset.files[idx][s .> α])
    end
    return keep
end

# One whole step (forward, loss, backward, ADAM(η) with β = (0.9, 0.999), ϵ = 1e-8) replayed as a
# captured hipGraph; the same kernels in the same order as train_loss + gradient! + update!
function train_step_graph!(m::HIPModel, x::ROCArray{Float32,5}, auto_loss, η)
    m.packed || repack!(m)
    m.step += 1; loss = ROCVector{Float32}(undef, 1)
    check(ccall((:md2_model_train_step_graph, lib), Cint,
                (Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Cfloat, Cint,
                 Ptr{Float32}, Ptr{Cvoid}),
                m.handle, x, ptr(auto_loss), m.m, m.v, η, m.step, loss, stream_ptr()))
    return loss
end

# ------------------------------------------------------------------------------------------------
# MINE plane rendering of the MPI mode (src/render.jl:21-114), forward only as upstream.  Same
# names and argument order as the reference; `pose` is a Pose(rvec (3,B), tvec (3,B)) and goes to
# the library as (6,B) = [B][6]; K / invK are host 3x3 matrices.
# ------------------------------------------------------------------------------------------------
pose6(pose) = ROCArray{Float32}(vcat(reshape(pose.rvec, 3, :), reshape(pose.tvec, 3, :)))

function get_src_xyz_from_plane_disparity(meshgrid_src_homo, mpi_disparity_src::ROCArray{Float32,2}, K_src_inv)
    _, W, H = size(meshgrid_src_homo)                  # create_meshgrid(H, W): the kernel's grid
    N, B = size(mpi_disparity_src); xyz = ROCArray{Float32}(undef, 3, W, H, N, B)
    iK = collect(rowmajor(K_src_inv))
    check(ccall((:md2_mine_src_xyz, lib), Cint,
                (Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                mpi_disparity_src, N, B, H, W, iK, xyz, stream_ptr()))
    return xyz
end

function get_tgt_xyz_from_plane_disparity(xyz_src::ROCArray{Float32,5}, pose)
    _, W, H, N, B = size(xyz_src); out = similar(xyz_src)
    check(ccall((:md2_mine_tgt_xyz, lib), Cint,
                (Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{Cvoid}),
                xyz_src, pose6(pose), N, B, H, W, out, stream_ptr()))
    return out
end

# sample(src (W,H,C,N*B), depth_src (N,B), pose, K, K_inv) -> (tgt, valid_mask (W*H, N*B))
function sample(src::ROCArray{Float32,4}, depth_src::ROCArray{Float32,2}, pose, K, K_inv)
    W, H, C, NB = size(src); N, B = size(depth_src)
    tgt = similar(src); valid = ROCArray{Float32}(undef, W * H, NB)
    k = collect(rowmajor(K)); ik = collect(rowmajor(K_inv))
    check(ccall((:md2_mine_sample, lib), Cint,
                (Ptr{Float32}, Cint, Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32},
                 Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                src, C, depth_src, pose6(pose), N, B, H, W, k, ik, tgt, valid, stream_ptr()))
    return tgt, valid .> 0
end

function plane_volume_rendering(rgb::ROCArray{Float32,5}, sigma::ROCArray{Float32,5}, xyz::ROCArray{Float32,5})
    W, H, _, N, B = size(rgb)
    rgb_out = ROCArray{Float32}(undef, W, H, 3, B)
    acc = ROCArray{Float32}(undef, W, H, 1, N, B); weights = similar(acc)
    check(ccall((:md2_plane_volume_rendering, lib), Cint,
                (Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32},
                 Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                rgb, sigma, xyz, N, B, H, W, rgb_out, acc, weights, stream_ptr()))
    return rgb_out, acc, weights
end

# one fused kernel: homography warp of rgb/sigma/xyz per plane + volume rendering + valid count
function render_tgt_rgb_depth(rgb::ROCArray{Float32,5}, sigma::ROCArray{Float32,5},
                              disparity_src::ROCArray{Float32,2}, xyz_tgt::ROCArray{Float32,5}, pose, K_inv, K)
    W, H, _, N, B = size(rgb)
    rgb_out = ROCArray{Float32}(undef, W, H, 3, B)
    depth = ROCArray{Float32}(undef, W, H, 1, N, B); mask = ROCArray{Float32}(undef, W, H, 1, 1, B)
    ik = collect(rowmajor(K_inv)); k = collect(rowmajor(K))
    check(ccall((:md2_render_tgt_rgb_depth, lib), Cint,
                (Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                 Ptr{Float32}, Cint, Cint, Cint, Cint, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Cvoid}),
                rgb, sigma, disparity_src, xyz_tgt, pose6(pose), ik, k, N, B, H, W, rgb_out, depth, mask,
                stream_ptr()))
    return rgb_out, depth, mask
end

# ------------------------------------------------------------------------------------------------
# Data parallel: one Julia process per GPU over the library's own RCCL communicator (SURVEY 8e;
# the reference's loop is scripts/script.jl:84-86).  Rank 0 writes the unique id to `idfile`,
# tagged with `run_id` -- a string unique to this launch that every rank gets from the launcher
# (e.g. the job id) -- and the other ranks accept only a file carrying their own tag, so a file
# left over from an earlier run can never hand them a stale id (ncclCommInitRank would hang).
# ------------------------------------------------------------------------------------------------
function comm_init(rank, nranks, device, idfile; run_id=get(ENV, "MD2_RUN_ID", ""), timeout_s=300)
    isempty(run_id) && error("comm_init: pass run_id (or set MD2_RUN_ID) unique to this launch")
    tag = Vector{UInt8}(run_id)
    id = zeros(UInt8, 128)
    if rank == 0
        check(ccall((:md2_comm_get_unique_id, lib), Cint, (Ptr{UInt8},), id))
        write(idfile * ".tmp", vcat(id, tag)); mv(idfile * ".tmp", idfile; force=true)
    else
        t0 = time()
        while true
            if isfile(idfile)
                b = read(idfile)
                if length(b) == 128 + length(tag) && b[129:end] == tag
                    id .= b[1:128]
                    break
                end
            end
            time() - t0 > timeout_s && error("comm_init: rank ", rank, " saw no id file ", idfile,
                                             " tagged ", run_id, " from rank 0 within ", timeout_s, " s")
            sleep(0.05)
        end
    end
    c = Ref{Ptr{Cvoid}}()
    check(ccall((:md2_comm_init, lib), Cint, (Cint, Cint, Ptr{UInt8}, Cint, Ref{Ptr{Cvoid}}),
                rank, nranks, id, device, c))
    return c[]
end

# forward + loss + backward with each bucket's RCCL all-reduce overlapped + ADAM (1/nranks)
function train_step_dp!(m::HIPModel, comm::Ptr{Cvoid}, x, auto_loss, η; β=(0.9f0, 0.999f0), ϵ=1f-8)
    m.packed || repack!(m)
    m.step += 1; loss = ROCVector{Float32}(undef, 1)
    check(ccall((:md2_model_train_step_dp, lib), Cint,
                (Ptr{Cvoid}, Ptr{Cvoid}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32}, Ptr{Float32},
                 Cfloat, Cfloat, Cfloat, Cfloat, Cint, Ptr{Float32}, Ptr{Cvoid}),
                m.handle, comm, x, ptr(auto_loss), m.m, m.v, η, β[1], β[2], ϵ, m.step, loss, stream_ptr()))
    return loss
end

# MPI mode: the disparity bins of the next train_loss, [batch][num_bins] on the device -- the
# uniformly_sample_disparity_from_linspace_bins draw of src/model.jl:17-21 (CUDA.rand there)
function set_disparity_bins!(m::HIPModel, bins::ROCArray{Float32,2})
    check(ccall((:md2_model_set_disparity_bins, lib), Cint, (Ptr{Cvoid}, Ptr{Float32}, Ptr{Cvoid}),
                m.handle, bins, stream_ptr()))
    return m
end

# ------------------------------------------------------------------------------------------------
# Data path (src/dtk.jl:29-46 Depth10k + FlipX, src/kitty.jl:45-61 KittyDataset): PNGs decoded on
# the host's cores into N0f8 bytes, widened to Float32 on the GPU
# ------------------------------------------------------------------------------------------------
function png_size(path::AbstractString)
    w, h, c = Ref{Cint}(0), Ref{Cint}(0), Ref{Cint}(0)
    check(ccall((:md2_png_info, lib), Cint, (Cstring, Ref{Cint}, Ref{Cint}, Ref{Cint}), path, w, h, c))
    return (w[], h[], c[])
end

function _to_device(bytes::Vector{UInt8}, dims)
    d8 = ROCArray(bytes)
    out = ROCArray{Float32}(undef, dims...)
    check(ccall((:md2_unorm8_to_float, lib), Cint, (Ptr{UInt8}, Ptr{Float32}, Clonglong, Ptr{Cvoid}),
                d8, out, length(bytes), stream_ptr()))
    return out
end

# Depth10k triplets (3W x H side-by-side RGB PNGs) -> x::(W, H, 3, 3, n) Float32 on the device
function load_triplets(paths::Vector{String}, width, height; flip=falses(length(paths)), threads=Threads.nthreads())
    n = length(paths)
    buf = Vector{UInt8}(undef, n * 3 * 3 * height * width)
    fl = UInt8.(flip)
    check(ccall((:md2_load_triplets_u8, lib), Cint,
                (Ptr{Cstring}, Cint, Cint, Cint, Ptr{UInt8}, Ptr{UInt8}, Cint),
                paths, n, width, height, fl, buf, threads))
    return _to_device(buf, (width, height, 3, 3, n))
end

# KittyDataset: paths[3i+k] = frame k of sample i (8-bit gray), imresize'd to (height, width)
function load_kitti(paths::Vector{String}, height, width; flip=falses(length(paths) ÷ 3), threads=Threads.nthreads())
    n = length(paths) ÷ 3
    buf = Vector{UInt8}(undef, n * 3 * height * width)
    fl = UInt8.(flip)
    check(ccall((:md2_load_kitti_u8, lib), Cint,
                (Ptr{Cstring}, Cint, Cint, Cint, Ptr{UInt8}, Ptr{UInt8}, Cint),
                paths, n, height, width, fl, buf, threads))
    return _to_device(buf, (width, height, 1, 3, n))
end

end # module
