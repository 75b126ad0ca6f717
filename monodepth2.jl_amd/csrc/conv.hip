// Implicit-GEMM convolution kernels for gfx950 (see conv.h).
//
// All three passes are one GEMM shape  C[M][N] = sum_k A[k][m] * B[k][n]  computed with the
// exact-fp32 MFMA v_mfma_f32_32x32x2_f32 (64 lanes: A[i=l&31][k=l>>5], B[k=l>>5][j=l&31]; C/D:
// col j = lane&31, row i = (r&3) + 8(r>>2) + 4(lane>>5)).  The N (lane) dimension is always the
// pixel or filter-column axis, so every epilogue store writes 32 consecutive floats per register.
//
//   forward : M = Cout, N = images*Ho*Wo,  K = Cin*KH*KW     A = packed W^T,  B = im2col(x)
//   dgrad   : M = Cin,  N = images*H*W,    K = Cout*KH*KW    A = packed W,    B = gather(dY)
//   wgrad   : M = Cout, N = Cin*KH*KW,     K = images*Ho*Wo  A = dY^T,        B = im2col(x)^T
//
// Tiles are staged global -> registers -> LDS (double buffered, one barrier per K step); the
// im2col / gather address maths runs on SALU (wave-uniform k decode) and VALU in the shadow of
// the 64-cycle f32 MFMAs.  Small-M / huge-K shapes (layer4, wgrad) use split-K slabs reduced by
// a second kernel that also applies the epilogue (deterministic, no atomics).
#include "conv.h"
#include "head.h"

namespace md2 {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int KPAD = 32;    // packed weight K padding
constexpr int MPAD = 128;   // packed weight M padding

static inline long round_up(long a, long b) { return (a + b - 1) / b * b; }

__device__ __forceinline__ int refl(int i, int n) { return i < 0 ? -i : (i >= n ? 2 * n - 2 - i : i); }

__device__ __forceinline__ float apply_act(float v, int act) {
  switch (act) {
    case ACT_RELU: return fmaxf(v, 0.f);
    case ACT_ELU: return v > 0.f ? v : expm1f(v);
    case ACT_SIGMOID: return 1.f / (1.f + expf(-v));
    default: return v;
  }
}

// ---------------------------------------------------------------------------------------------
// weight packing
// ---------------------------------------------------------------------------------------------
// forward:  Wt[k][m] = W[m][c][tap]   ([Kpad][Mpad]);   dgrad: Wd[k][ci] = W[co][ci][tap]
// ([Kdpad][Cinpad]); k = tap*C + c (tap-major) or c*KK + tap, C = Cin (forward) / Cout (dgrad)
struct PackOne {
  const float* w;
  float* out;
  int mode, tap, layout, Cout, Cin, KK, Kpad, Mpad;
};

__device__ __forceinline__ long packed_index(int k, int m, int layout, int Mpad) {
  return layout ? ((long)(k >> 4) * Mpad + m) * 16 + (k & 15) : (long)k * Mpad + m;
}

// single-operand pack (op-level ABI): destination order, writes the zero padding too
__global__ __launch_bounds__(256) void pack_one_kernel(PackOne j) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= (long)j.Kpad * j.Mpad) return;
  int k, m;
  if (j.layout) {
    const long chunk = (long)j.Mpad * 16;
    const int kc = (int)(idx / chunk);
    const int r = (int)(idx - kc * chunk);
    m = r >> 4;
    k = kc * 16 + (r & 15);
  } else {
    k = (int)(idx / j.Mpad);
    m = (int)(idx % j.Mpad);
  }
  const int C = j.mode == 0 ? j.Cin : j.Cout;     // reduction channels
  const int Mr = j.mode == 0 ? j.Cout : j.Cin;    // rows
  float v = 0.f;
  if (k < C * j.KK && m < Mr) {
    int c, tap;
    if (j.tap) {
      tap = k / C;
      c = k - tap * C;
    } else {
      c = k / j.KK;
      tap = k - c * j.KK;
    }
    const long co = j.mode == 0 ? m : c, ci = j.mode == 0 ? c : m;
    v = j.w[(co * j.Cin + ci) * j.KK + tap];
  }
  j.out[idx] = v;
}

size_t conv_fwd_packed_elems(const ConvShape& s) {
  return (size_t)round_up((long)s.Cin * s.KH * s.KW, KPAD) * round_up(s.Cout, MPAD);
}
size_t conv_dgrad_packed_elems(const ConvShape& s) {
  return (size_t)round_up((long)s.Cout * s.KH * s.KW, KPAD) * round_up(s.Cin, MPAD);
}

static int pack_single(const ConvShape& s, int mode, const float* w, float* packed, hipStream_t st) {
  PackOne j{};
  j.w = w;
  j.out = packed;
  j.mode = mode;
  j.tap = conv_tap_major(s, mode) ? 1 : 0;
  j.layout = conv_px2_used(s, mode) ? 1 : 0;
  j.Cout = s.Cout;
  j.Cin = s.Cin;
  j.KK = s.KH * s.KW;
  j.Kpad = (int)(mode == 0 ? round_up((long)s.Cin * j.KK, KPAD) : round_up((long)s.Cout * j.KK, KPAD));
  j.Mpad = (int)(mode == 0 ? round_up(s.Cout, MPAD) : round_up(s.Cin, MPAD));
  hipLaunchKernelGGL(pack_one_kernel, dim3(cdiv((long)j.Kpad * j.Mpad, 256)), dim3(256), 0, st, j);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}
int conv_pack_fwd(const ConvShape& s, const float* w, float* packed, hipStream_t st) {
  return pack_single(s, 0, w, packed, st);
}
int conv_pack_dgrad(const ConvShape& s, const float* w, float* packed, hipStream_t st) {
  return pack_single(s, 1, w, packed, st);
}

PackJob conv_pack_job(const ConvShape& s, const float* w, float* out_f, float* out_d) {
  PackJob j{};
  j.w = w;
  j.Cout = s.Cout;
  j.Cin = s.Cin;
  j.KK = s.KH * s.KW;
  j.f = PackDst{out_f, conv_tap_major(s, 0) ? 1 : 0, conv_px2_used(s, 0) ? 1 : 0,
                (int)round_up(s.Cout, MPAD)};
  j.d = PackDst{out_d, conv_tap_major(s, 1) ? 1 : 0, conv_px2_used(s, 1) ? 1 : 0,
                (int)round_up(s.Cin, MPAD)};
  return j;
}

long conv_pack_job_blocks(const PackJob& j) { return cdiv((long)j.Cout * j.Cin * j.KK, 256); }

// Source-ordered: consecutive threads read consecutive weights (coalesced, each weight read
// once); the two scattered writes of a block land in a few packed rows that L2 merges into
// full lines.  Destination padding is never touched (zeroed at allocation).
__global__ __launch_bounds__(256) void pack_batch_kernel(const PackJob* __restrict__ jobs, int njobs) {
  __shared__ int s_job;
  if (threadIdx.x == 0) {
    int lo = 0, hi = njobs - 1;
    while (lo < hi) {
      const int mid = (lo + hi + 1) >> 1;
      if (jobs[mid].block_begin <= (long)blockIdx.x) lo = mid; else hi = mid - 1;
    }
    s_job = lo;
  }
  __syncthreads();
  const PackJob& j = jobs[__builtin_amdgcn_readfirstlane(s_job)];
  const unsigned e = (unsigned)(blockIdx.x - j.block_begin) * 256u + threadIdx.x;
  const unsigned KK = (unsigned)j.KK, Cin = (unsigned)j.Cin;
  if (e >= (unsigned)j.Cout * Cin * KK) return;
  const float v = j.w[e];
  const unsigned row = e / KK;
  const int tap = (int)(e - row * KK);
  const int co = (int)(row / Cin);
  const int ci = (int)(row - (unsigned)co * Cin);
  if (j.f.out) {
    const int k = j.f.tap ? tap * j.Cin + ci : ci * j.KK + tap;
    j.f.out[packed_index(k, co, j.f.layout, j.f.Mpad)] = v;
  }
  if (j.d.out) {
    const int k = j.d.tap ? tap * j.Cout + co : co * j.KK + tap;
    j.d.out[packed_index(k, ci, j.d.layout, j.d.Mpad)] = v;
  }
}

int conv_pack_batch(const PackJob* dev_jobs, int njobs, long total_blocks, hipStream_t st) {
  if (njobs == 0) return MD2_OK;
  hipLaunchKernelGGL(pack_batch_kernel, dim3(total_blocks), dim3(256), 0, st, dev_jobs, njobs);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// ---------------------------------------------------------------------------------------------
// kernel arguments
// ---------------------------------------------------------------------------------------------
struct GemmDims {
  int M;
  long N;       // pixels (fwd/dgrad) or filter columns (wgrad)
  int K;        // reduction length (fwd/dgrad); wgrad: pixels (long fits int here)
  int kper;     // K elements per split (multiple of BK)
  int Mpad;     // packed A leading dimension (fwd/dgrad)
};

struct ConvArgs {
  GemmDims g;
  int Cin, H, W, Cout, Ho, Wo, stride, pad;
  long HW, HoWo;
  FastDiv fd_pix;    // pixels per image of the N axis (Ho*Wo fwd/wgrad, H*W dgrad)
  FastDiv fd_row;    // row length of the N axis (Wo fwd/wgrad, W dgrad)
  FastDiv fd_bdiv;
  TensorIn in;
  const float* A;    // packed weights (fwd/dgrad)
  const float* dy;   // dgrad / wgrad
  TensorOut out;
  float* slab;       // split-K partials [splits][M][N] or nullptr
  // byte extents of the buffer resources (raw buffer loads: an offset past the extent reads 0,
  // which implements the zero padding of the gathers without branches)
  uint32_t A_bytes, b0_bytes, b1_bytes;
  uint32_t HW4, HoWo4;   // channel strides in bytes (scalar soffset steps of the tap-major gathers)
  // stride-2 dgrad by output-parity class (tap-major only): the N axis enumerates the input
  // pixels (ph_y0 + 2j, ph_x0 + 2i) of one class (fd_pix / fd_row are the class extents) and K
  // runs over that class's taps ph_taps[0..ntaps) only
  int ph_y0, ph_x0;
  int ph_taps[16];       // <= ceil(7/2)^2 taps per class
};

// (image, pixel-in-plane) of N-axis element nn for fwd / dgrad outputs
__device__ __forceinline__ void out_pixel(const ConvArgs& a, bool phase, long nn, int& img, long& pix,
                                          long& plane) {
  img = (int)fdiv((uint32_t)nn, a.fd_pix);
  const long r = nn - (long)img * a.fd_pix.d;
  if (phase) {
    const int jy = (int)fdiv((uint32_t)r, a.fd_row);
    const int jx = (int)(r - (long)jy * a.fd_row.d);
    pix = (long)(a.ph_y0 + 2 * jy) * a.W + a.ph_x0 + 2 * jx;
    plane = a.HW;
  } else {
    pix = r;
    plane = a.fd_pix.d;
  }
}

template <int TM, int TN, int BK>
__device__ __forceinline__ void mma_chunk(const float* __restrict__ As, int lda,
                                          const float* __restrict__ Bs, int ldb, int am0, int bn0,
                                          int lane, f32x16 (&acc)[TM][TN]) {
  const int kh = lane >> 5, l = lane & 31;
  // fragments of k-step kk+1 are read while the MFMAs of kk issue (register double buffer;
  // fully unrolled so every index is static)
  float a[2][TM], b[2][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i) a[0][i] = As[kh * lda + am0 + i * 32 + l];
#pragma unroll
  for (int j = 0; j < TN; ++j) b[0][j] = Bs[kh * ldb + bn0 + j * 32 + l];
#pragma unroll
  for (int kk = 0; kk < BK / 2; ++kk) {
    const int cur = kk & 1, nxt = cur ^ 1;
    if (kk + 1 < BK / 2) {
#pragma unroll
      for (int i = 0; i < TM; ++i) a[nxt][i] = As[(2 * kk + 2 + kh) * lda + am0 + i * 32 + l];
#pragma unroll
      for (int j = 0; j < TN; ++j) b[nxt][j] = Bs[(2 * kk + 2 + kh) * ldb + bn0 + j * 32 + l];
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[cur][i], b[cur][j], acc[i][j], 0, 0, 0);
  }
}

// Epilogue of one accumulator element (m, n) for the NCHW-style outputs of fwd / dgrad.
__device__ __forceinline__ void store_out(const TensorOut& o, int m, int img, long pix, long HoWo,
                                          float v) {
  if (o.bias) v += o.bias[m];
  v = apply_act(v, o.act);
  float* dst = (m < o.c0) ? o.p0 + (long)img * o.bs0 + (long)m * HoWo + pix
                          : o.p1 + (long)img * o.bs1 + (long)(m - o.c0) * HoWo + pix;
  if (o.accumulate)
    *dst += v;
  else
    *dst = v;
}

#include "conv_px.inc"
#include "conv_px2.inc"

// split-K reduction + epilogue for fwd / dgrad
__global__ __launch_bounds__(256) void splitk_reduce_px_kernel(ConvArgs a, int splits, int phase) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long total = (long)a.g.M * a.g.N;
  if (idx >= total) return;
  const int m = (int)(idx / a.g.N);
  const long nn = idx - (long)m * a.g.N;
  float v = 0.f;
  for (int s = 0; s < splits; ++s) v += a.slab[(long)s * total + idx];
  int img;
  long pix, plane;
  out_pixel(a, phase != 0, nn, img, pix, plane);
  store_out(a.out, m, img, pix, plane, v);
}

// ---------------------------------------------------------------------------------------------
// wgrad kernel: lanes along the pixel (K) axis for both operands, transposed into LDS
// ---------------------------------------------------------------------------------------------
template <int BM, int BN, int BK, int WM, int WN, int KH, int KW, int S, int RFL>
__global__ __launch_bounds__(256) void conv_wgrad_kernel(ConvArgs a) {
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
  constexpr int KK = KH * KW;
  constexpr int RP = 256 / BK;          // rows per pass
  constexpr int A_EL = BM / RP, B_EL = BN / RP;
  constexpr int LDA = BM + 1, LDB = BN + 1;
  static_assert(A_EL >= 1 && B_EL >= 1, "tile");
  __shared__ float As[2][BK][LDA];
  __shared__ float Bs[2][BK][LDB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.y * BM;
  const int n0 = blockIdx.x * BN;
  const long kbeg = (long)blockIdx.z * a.g.kper;
  const long Ktot = a.g.K;
  const long kend = min(Ktot, kbeg + (long)a.g.kper);
  const int nk = (int)((kend - kbeg + BK - 1) / BK);
  const int kl = tid % BK;
  const int rg = tid / BK;

  // per-thread filter columns of B (fixed for the whole kernel)
  float areg[A_EL], breg[B_EL];

  auto load = [&](long k0) {
    const long p = k0 + kl;
    const bool pv = p < kend;
    int img = 0, oy = 0, ox = 0;
    if (pv) {
      img = (int)fdiv((uint32_t)p, a.fd_pix);
      const int pix = (int)(p - (long)img * a.fd_pix.d);
      oy = (int)fdiv((uint32_t)pix, a.fd_row);
      ox = pix - oy * (int)a.fd_row.d;
    }
    const float* dyb = a.dy + (long)img * a.Cout * a.HoWo + (long)oy * a.Wo + ox;
#pragma unroll
    for (int j = 0; j < A_EL; ++j) {
      const int m = m0 + rg + j * RP;
      areg[j] = (pv && m < a.g.M) ? dyb[(long)m * a.HoWo] : 0.f;
    }
    const int q = (int)fdiv((uint32_t)img, a.fd_bdiv);
    const float* b0 = a.in.p0 + (long)(img - q * (int)a.fd_bdiv.d) * a.in.bs0 + (long)q * a.in.bhi;
    const float* b1 = a.in.p1 ? a.in.p1 + (long)img * a.in.bs1 : nullptr;
    const int py = oy * S - a.pad, px = ox * S - a.pad;
#pragma unroll
    for (int j = 0; j < B_EL; ++j) {
      const int nidx = n0 + rg + j * RP;
      float v = 0.f;
      if (pv && nidx < a.g.N) {
        const int c = nidx / KK;
        const int r = nidx - c * KK;
        const int kh = r / KW, kw = r - (r / KW) * KW;
        int iy = py + kh, ix = px + kw;
        bool ok = true;
        if (RFL) {
          iy = refl(iy, a.H);
          ix = refl(ix, a.W);
        } else {
          ok = (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;
        }
        const float* src = (c < a.in.c0) ? b0 + (long)c * a.HW : b1 + (long)(c - a.in.c0) * a.HW;
        if (ok) v = src[iy * a.W + ix];
      }
      breg[j] = v;
    }
  };
  auto store_tiles = [&](int buf) {
#pragma unroll
    for (int j = 0; j < A_EL; ++j) As[buf][kl][rg + j * RP] = areg[j];
#pragma unroll
    for (int j = 0; j < B_EL; ++j) Bs[buf][kl][rg + j * RP] = breg[j];
  };

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    load(kbeg);
    store_tiles(0);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) load(kbeg + (long)(t + 1) * BK);
    mma_chunk<TM, TN, BK>(&As[cur][0][0], LDA, &Bs[cur][0][0], LDB, wm * TM * 32, wn * TN * 32, lane, acc);
    if (t + 1 < nk) store_tiles(cur ^ 1);
    __syncthreads();
  }

  float* sl = a.slab + (long)blockIdx.z * a.g.M * a.g.N;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const long nn = n0 + wn * TN * 32 + j * 32 + (lane & 31);
    if (nn >= a.g.N) continue;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < a.g.M) sl[(long)m * a.g.N + nn] = acc[i][j][r];
      }
  }
}

// tap-major wgrad: filter columns n = tap*Cin + c.  A block covers TT = BN/CW consecutive taps
// x CW channels (CW | Cin, and CW | the concat split, so the block reads one tensor): row j of a
// thread is tap (RP*j)/CW and channel (RP*j)%CW + rg, both compile-time up to the block base.
// Per K chunk each thread computes one gather offset per tap (TT of them); every element is then
// a buffer load with that offset and a scalar channel soffset -- no VALU per element.  The slab
// is written in (m, n) tap-major order; the final reduction permutes to [Cout][Cin][KH][KW].
template <int BM, int BN, int BK, int WM, int WN, int KH, int KW, int S, int RFL, int CW>
__global__ __launch_bounds__(256) void conv_wgrad_tap_kernel(ConvArgs a) {
  constexpr int TM = BM / (32 * WM), TN = BN / (32 * WN);
  constexpr int KK = KH * KW;
  constexpr int RP = 256 / BK;          // rows per pass
  constexpr int A_EL = BM / RP, B_EL = BN / RP;
  constexpr int TT = BN / CW;           // taps per block
  constexpr int LDA = BM + 1, LDB = BN + 1;
  static_assert(A_EL >= 1 && B_EL >= 1 && TT >= 1 && CW % RP == 0, "tile");
  __shared__ float As[2][BK][LDA];
  __shared__ float Bs[2][BK][LDB];

  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;
  const int m0 = blockIdx.y * BM;
  const int ncb = a.Cin / CW;
  const int tb = (int)blockIdx.x / ncb * TT;           // first tap of the block
  const int cbk = ((int)blockIdx.x % ncb) * CW;        // first channel of the block
  const int kbeg = blockIdx.z * a.g.kper;
  const int kend = min(a.g.K, kbeg + a.g.kper);
  const int nk = (kend - kbeg + BK - 1) / BK;
  const int kl = tid % BK;
  const int rg = tid / BK;
  const int mlim = a.g.M - m0 - rg;     // row j of dY valid iff RP*j < mlim

  const bool sec = cbk >= a.in.c0;      // block-uniform concat side
  const __amdgpu_buffer_rsrc_t rdy = make_rsrc(a.dy, a.A_bytes);
  const __amdgpu_buffer_rsrc_t rx = sec ? make_rsrc(a.in.p1, a.b1_bytes) : make_rsrc(a.in.p0, a.b0_bytes);
  const uint32_t cso = (uint32_t)(sec ? cbk - a.in.c0 : cbk) * a.HW4;

  float areg[A_EL], breg[B_EL];

  // all offsets in 32 bits: every extent is < 2 GB (checked on the host)
#define MD2_W_LOAD(K0)                                                                            \
  {                                                                                               \
    const int p = (K0) + kl;                                                                      \
    const bool pv = p < kend;                                                                     \
    const uint32_t pc = (uint32_t)(pv ? p : kbeg);                                                \
    const uint32_t img = fdiv(pc, a.fd_pix);                                                      \
    const uint32_t pix = pc - img * a.fd_pix.d;                                                   \
    const uint32_t oy = fdiv(pix, a.fd_row);                                                      \
    const uint32_t ox = pix - oy * a.fd_row.d;                                                    \
    const uint32_t va = pv ? ((img * (uint32_t)a.Cout + rg) * (uint32_t)a.HoWo + pix) * 4u : OOB; \
    _Pragma("unroll") for (int j = 0; j < A_EL; ++j)                                              \
      areg[j] = bload_s(rdy, RP * j < mlim ? va : OOB, (uint32_t)(m0 + RP * j) * a.HoWo4);        \
    uint32_t vb;                                                                                  \
    if (sec) {                                                                                    \
      vb = (img * (uint32_t)a.in.bs1 + rg * (uint32_t)a.HW) * 4u;                                 \
    } else {                                                                                      \
      const uint32_t q = fdiv(img, a.fd_bdiv);                                                    \
      vb = ((img - q * a.fd_bdiv.d) * (uint32_t)a.in.bs0 + q * (uint32_t)a.in.bhi +               \
            rg * (uint32_t)a.HW) * 4u;                                                            \
    }                                                                                             \
    const int py = (int)oy * S - a.pad, px = (int)ox * S - a.pad;                                 \
    uint32_t vt[TT];                                                                              \
    _Pragma("unroll") for (int t = 0; t < TT; ++t) {                                              \
      const int tap = tb + t;                                                                     \
      const int kh = tap / KW, kw = tap - (tap / KW) * KW;                                        \
      int iy = py + kh, ix = px + kw;                                                             \
      bool ok;                                                                                    \
      if (RFL) {                                                                                  \
        iy = refl(iy, a.H);                                                                       \
        ix = refl(ix, a.W);                                                                       \
        ok = pv;                                                                                  \
      } else {                                                                                    \
        ok = pv && (unsigned)iy < (unsigned)a.H && (unsigned)ix < (unsigned)a.W;                  \
      }                                                                                           \
      vt[t] = (ok && tap < KK) ? vb + (uint32_t)(iy * a.W + ix) * 4u : OOB;                       \
    }                                                                                             \
    _Pragma("unroll") for (int j = 0; j < B_EL; ++j)                                              \
      breg[j] = bload_s(rx, vt[(RP * j) / CW], cso + (uint32_t)((RP * j) % CW) * a.HW4);         \
  }
#define MD2_W_STORE(BUF)                                                                          \
  _Pragma("unroll") for (int j = 0; j < A_EL; ++j) As[BUF][kl][rg + j * RP] = areg[j];            \
  _Pragma("unroll") for (int j = 0; j < B_EL; ++j) Bs[BUF][kl][rg + j * RP] = breg[j];

  f32x16 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[i][j][r] = 0.f;

  if (nk > 0) {
    MD2_W_LOAD(kbeg);
    MD2_W_STORE(0);
  }
  __syncthreads();
  for (int t = 0; t < nk; ++t) {
    const int cur = t & 1;
    if (t + 1 < nk) MD2_W_LOAD(kbeg + (t + 1) * BK);
    mma_chunk<TM, TN, BK>(&As[cur][0][0], LDA, &Bs[cur][0][0], LDB, wm * TM * 32, wn * TN * 32, lane, acc);
    if (t + 1 < nk) {
      MD2_W_STORE(cur ^ 1);
    }
    __syncthreads();
  }
#undef MD2_W_LOAD
#undef MD2_W_STORE

  float* sl = a.slab + (long)blockIdx.z * a.g.M * a.g.N;
#pragma unroll
  for (int j = 0; j < TN; ++j) {
    const int nl = wn * TN * 32 + j * 32 + (lane & 31);
    const int tap = tb + nl / CW;
    if (tap >= KK) continue;
    const long nn = (long)tap * a.Cin + cbk + nl % CW;
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int m = m0 + wm * TM * 32 + i * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
        if (m < a.g.M) sl[(long)m * a.g.N + nn] = acc[i][j][r];
      }
  }
}

// split-K slab reduction for wgrad, two stages for parallelism: stage 1 sums split groups
// (group g takes splits g, g+G, ...) into part[G][total]; stage 2 sums the G partials.
constexpr int WRED_GROUPS = 32;

__global__ __launch_bounds__(256) void splitk_reduce_w1_kernel(const float* __restrict__ slab,
                                                               int splits, long total, int G,
                                                               float* __restrict__ part) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  const int g = blockIdx.y;
  float v0 = 0.f, v1 = 0.f;
  int s = g;
  for (; s + G < splits; s += 2 * G) {
    v0 += slab[(long)s * total + idx];
    v1 += slab[(long)(s + G) * total + idx];
  }
  if (s < splits) v0 += slab[(long)s * total + idx];
  part[(long)g * total + idx] = v0 + v1;
}

// stage 2; tapc > 0: slab columns are tap-major (n = tap*Cin + c, Cin = tapc) and are written
// to the [Cout][Cin][KK] parameter layout
__global__ __launch_bounds__(256) void splitk_reduce_w2_kernel(const float* __restrict__ part,
                                                               int G, long total,
                                                               float* __restrict__ dw, int acc,
                                                               int ncols, int tapc, int KK) {
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  if (idx >= total) return;
  float v = 0.f;
  for (int g = 0; g < G; ++g) v += part[(long)g * total + idx];
  long o = idx;
  if (tapc > 0) {
    const long m = idx / ncols;
    const int n = (int)(idx - m * ncols);
    const int tp = n / tapc, c = n - tp * tapc;
    o = m * ncols + (long)c * KK + tp;
  }
  if (acc)
    dw[o] += v;
  else
    dw[o] = v;
}

// bias gradient db[c] = sum over images and pixels of dY[img][c][:], two stages:
// grid (C, parts) partial sums over contiguous slices of the N*HW elements, then per channel.
__global__ __launch_bounds__(256) void bias_grad_partial_kernel(const float* __restrict__ dy, int C,
                                                                long HW, long total, int parts,
                                                                float* __restrict__ part) {
  __shared__ float red[4];
  const int c = blockIdx.x, p = blockIdx.y;
  const long beg = total * p / parts, end = total * (p + 1) / parts;
  float s = 0.f;
  for (long e = beg + threadIdx.x; e < end; e += 256) {
    const long img = e / HW, pix = e - img * HW;
    s += dy[(img * C + c) * HW + pix];
  }
  float v[1] = {s};
  block_sum256<1>(v, red);
  if (threadIdx.x == 0) part[(long)c * parts + p] = v[0];
}

__global__ void bias_grad_final_kernel(const float* __restrict__ part, int C, int parts,
                                       float* __restrict__ db, int acc) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float s = 0.f;
  for (int p = 0; p < parts; ++p) s += part[(long)c * parts + p];
  if (acc)
    db[c] += s;
  else
    db[c] = s;
}

static int bias_parts(int C, long total) {
  return (int)std::max(1L, std::min((long)std::max(1, 1024 / C), total / 4096 + 1));
}

__global__ __launch_bounds__(256) void act_backward_kernel(const float* __restrict__ out,
                                                           const float* __restrict__ dout,
                                                           float* __restrict__ dpre, long n,
                                                           int act) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float o = out[i], g = dout[i];
  float d;
  switch (act) {
    case ACT_RELU: d = o > 0.f ? g : 0.f; break;
    case ACT_ELU: d = o > 0.f ? g : g * (o + 1.f); break;      // elu'(x) = exp(x) = out + 1
    case ACT_SIGMOID: d = g * o * (1.f - o); break;
    default: d = g;
  }
  dpre[i] = d;
}

// ---------------------------------------------------------------------------------------------
// host side: tile selection, split-K planning, dispatch
// ---------------------------------------------------------------------------------------------
namespace {

constexpr int TARGET_BLOCKS = 1536;  // ~6 blocks (waves per SIMD) per CU on 256 CUs

enum TileCfg { T128x128 = 0, T64x256 = 1, T32x256 = 2, T64x128 = 3, T128x64 = 4, T64x64 = 5, T32x128 = 6 };
const int TILE_BM[] = {128, 64, 32, 64, 128, 64, 32};
const int TILE_BN[] = {128, 256, 256, 128, 64, 64, 128};

// debugging / tuning overrides of the planner (read once): MD2_PX_TILE=<TileCfg>,
// MD2_PX_TARGET=<target blocks for the split-K choice>
int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  return e ? atoi(e) : dflt;
}

struct Plan {
  int tile;
  int BM, BN, BK;
  int splits;
  int kper;
};

Plan plan_px(int M, long N, int K, bool bk32_ok = false) {
  // Small tiles, many blocks: at B=12 the GEMMs are ~0.5 chip of 128x128 tiles; 64x64 tiles
  // (30 VGPR + 16 AGPR, 8 waves/SIMD) with ~1536 blocks keep 4-6 waves per SIMD in flight and
  // ran 10-50% faster than 128x128 / 64x256 on every encoder shape (tools/sweep_px.sh, r01).
  static const int tile_override = env_int("MD2_PX_TILE", -1);
  static const int target = env_int("MD2_PX_TARGET", TARGET_BLOCKS);
  Plan p{};
  p.tile = M > 32 ? T64x64 : T32x128;
  if (tile_override >= 0 && tile_override <= T32x128 &&
      ((M > 32 && TILE_BM[tile_override] >= 64) || (M <= 32 && TILE_BM[tile_override] == 32)))
    p.tile = tile_override;
  p.BM = TILE_BM[p.tile];
  p.BN = TILE_BN[p.tile];
  static const int bk_override = env_int("MD2_PX_BK", 16);
  p.BK = (bk_override == 32 && bk32_ok) ? 32 : 16;
  if (K <= 0) {                // a parity class without taps: the kernel only writes zeros
    p.splits = 1;
    p.kper = p.BK;
    return p;
  }
  const long tiles = (long)cdiv(M, p.BM) * cdiv(N, p.BN);
  int splits = 1;
  while (tiles * splits * 2 <= target && K / (splits * 2) >= 8 * p.BK) splits *= 2;
  p.kper = (int)round_up(cdiv(K, splits), p.BK);
  p.splits = cdiv(K, p.kper);
  return p;
}

// wgrad tiles (BM x BN, 4 waves as WM x WN); columns are tap-major (tap groups x CW channels)
enum WTileCfg { W64x128 = 0, W32x256 = 1, W64x64 = 2, W32x128 = 3 };
const int WT_BM[] = {64, 32, 64, 32};
const int WT_BN[] = {128, 256, 64, 128};

struct WPlan {
  int tile, BM, BN;
  int cw;          // channels per tap block (0: channel-major kernel)
  long ntiles_n;   // column tiles
  int splits, kper;
};

// channels per tap block of the tap-major wgrad: largest of 128/64/32/16 (<= BN) dividing Cin and
// the concat split
int wgrad_cw(const ConvShape& s, int c0, int BN) {
  for (int cw = 128; cw >= 16; cw /= 2)
    if (cw <= BN && s.Cin % cw == 0 && (c0 >= s.Cin || c0 % cw == 0)) return cw;
  return 0;
}

WPlan plan_wgrad(const ConvShape& s, int c0) {
  static const int tile_override = env_int("MD2_W_TILE", -1);
  static const int target = env_int("MD2_W_TARGET", 0);
  WPlan p{};
  const int M = s.Cout;
  const int KK = s.KH * s.KW;
  auto ntiles = [&](int tile, int& cw) {
    cw = conv_tap_major(s, 2) ? wgrad_cw(s, c0, WT_BN[tile]) : 0;
    const long nt = cw ? (long)cdiv(KK, WT_BN[tile] / cw) * (s.Cin / cw) : cdiv((long)s.Cin * KK, WT_BN[tile]);
    return (long)cdiv(M, WT_BM[tile]) * nt;
  };
  // M <= 32: 32x128 (1024 blocks); else 64x128 with split-K to ~512 blocks, or 64x64 when the
  // grid is already >= 256 tiles without splitting (tools/sweep_w.sh, r01)
  int tgt = 512;
  if (M <= 32) {
    p.tile = W32x128;
    tgt = 1024;
  } else {
    int cw;
    p.tile = ntiles(W64x128, cw) >= 256 ? W64x64 : W64x128;
    if (p.tile == W64x64) tgt = 1024;
  }
  if (tile_override >= 0 && tile_override <= W32x128) p.tile = tile_override;
  if (target > 0) tgt = target;
  p.BM = WT_BM[p.tile];
  p.BN = WT_BN[p.tile];
  const long tiles = ntiles(p.tile, p.cw);
  p.ntiles_n = tiles / cdiv(M, p.BM);
  const long K = (long)s.N * s.Ho * s.Wo;
  const int BK = 32;
  long splits = std::max(1L, (long)tgt / tiles);
  splits = std::min(splits, std::max(1L, K / (8 * BK)));
  p.kper = (int)round_up((K + splits - 1) / splits, BK);
  p.splits = (int)((K + p.kper - 1) / p.kper);
  return p;
}

void fill_common(ConvArgs& a, const ConvShape& s) {
  a.Cin = s.Cin; a.H = s.H; a.W = s.W; a.Cout = s.Cout; a.Ho = s.Ho; a.Wo = s.Wo;
  a.stride = s.stride; a.pad = s.pad;
  a.HW = (long)s.H * s.W;
  a.HoWo = (long)s.Ho * s.Wo;
  a.HW4 = (uint32_t)(a.HW * 4);
  a.HoWo4 = (uint32_t)(a.HoWo * 4);
}

int check_shape(const ConvShape& s) {
  MD2_CHECK_ARG(s.N > 0 && s.Cin > 0 && s.Cout > 0 && s.H > 0 && s.W > 0, "conv dims");
  MD2_CHECK_ARG(s.KH == s.KW && (s.KH == 1 || s.KH == 3 || s.KH == 7), "kernel size 1/3/7");
  MD2_CHECK_ARG(s.stride == 1 || s.stride == 2, "stride 1/2");
  MD2_CHECK_ARG(s.Ho == (s.H + 2 * s.pad - s.KH) / s.stride + 1 &&
                    s.Wo == (s.W + 2 * s.pad - s.KW) / s.stride + 1, "output size");
  MD2_CHECK_ARG(!s.reflect || (s.KH == 3 && s.stride == 1 && s.pad == 1 && s.H >= 2 && s.W >= 2),
                "reflect padding needs 3x3/1 pad 1");
  MD2_CHECK_ARG((long)s.N * s.H * s.W < (1L << 31) && (long)s.N * s.Ho * s.Wo < (1L << 31),
                "pixel count");
  return MD2_OK;
}

// (KH, S, RFL) combos instantiated
#define MD2_CONV_COMBOS(X) X(1, 1, 0) X(1, 2, 0) X(3, 1, 0) X(3, 1, 1) X(3, 2, 0) X(7, 2, 0)

template <int MODE, int BM, int BN, int WM, int WN>
int launch_px_tile(const ConvShape& s, const ConvArgs& a, bool tap, int bk, dim3 grid, hipStream_t st) {
  const bool v2 = conv_px2_used(s, MODE);
#define MD2_PX_CASE(KS, SS, RR)                                                                  \
  if (s.KH == KS && s.stride == SS && s.reflect == RR) {                                         \
    if constexpr (BM >= 64 && BN % 64 == 0) {                                                    \
      if (v2) {                                                                                  \
        hipLaunchKernelGGL((conv_px2_kernel<MODE, BM, BN, WM, WN, KS, KS, SS, RR>), grid,        \
                           dim3(256), 0, st, a);                                                 \
        MD2_LAUNCH_CHECK();                                                                      \
        return MD2_OK;                                                                           \
      }                                                                                          \
    }                                                                                            \
    if (v2) {                                                                                    \
      set_error("conv: k-contiguous kernel needs a tile with BM >= 64");                         \
      return MD2_EINVAL;                                                                         \
    }                                                                                            \
    if (tap && bk == 32)                                                                         \
      hipLaunchKernelGGL((conv_px_kernel<MODE, 1, BM, BN, 32, WM, WN, KS, KS, SS, RR>), grid,    \
                         dim3(256), 0, st, a);                                                   \
    else if (tap)                                                                                \
      hipLaunchKernelGGL((conv_px_kernel<MODE, 1, BM, BN, 16, WM, WN, KS, KS, SS, RR>), grid,    \
                         dim3(256), 0, st, a);                                                   \
    else                                                                                         \
      hipLaunchKernelGGL((conv_px_kernel<MODE, 0, BM, BN, 16, WM, WN, KS, KS, SS, RR>), grid,    \
                         dim3(256), 0, st, a);                                                   \
    MD2_LAUNCH_CHECK();                                                                          \
    return MD2_OK;                                                                               \
  }
  MD2_CONV_COMBOS(MD2_PX_CASE)
#undef MD2_PX_CASE
  set_error("conv: unsupported (kernel, stride, padding) combination");
  return MD2_ENOTSUP;
}

template <int MODE>
int launch_px(const ConvShape& s, ConvArgs& a, const Plan& p, ConvWorkspace ws, hipStream_t st) {
  a.g.kper = p.kper;
  a.slab = nullptr;
  if (p.splits > 1) {
    const size_t need = (size_t)p.splits * a.g.M * a.g.N * sizeof(float);
    MD2_CHECK_ARG(ws.ptr && ws.bytes >= need, "conv split-K workspace too small");
    a.slab = (float*)ws.ptr;
  }
  dim3 grid(cdiv(a.g.N, p.BN), cdiv(a.g.M, p.BM), p.splits);
  const bool tap = conv_tap_major(s, MODE);
  int rc;
  switch (p.tile) {
    case T128x128: rc = launch_px_tile<MODE, 128, 128, 2, 2>(s, a, tap, p.BK, grid, st); break;
    case T64x256: rc = launch_px_tile<MODE, 64, 256, 1, 4>(s, a, tap, p.BK, grid, st); break;
    case T64x128: rc = launch_px_tile<MODE, 64, 128, 2, 2>(s, a, tap, p.BK, grid, st); break;
    case T128x64: rc = launch_px_tile<MODE, 128, 64, 2, 2>(s, a, tap, p.BK, grid, st); break;
    case T64x64: rc = launch_px_tile<MODE, 64, 64, 2, 2>(s, a, tap, p.BK, grid, st); break;
    case T32x128: rc = launch_px_tile<MODE, 32, 128, 1, 4>(s, a, tap, p.BK, grid, st); break;
    default: rc = launch_px_tile<MODE, 32, 256, 1, 4>(s, a, tap, p.BK, grid, st); break;
  }
  if (rc) return rc;
  if (p.splits > 1) {
    const long total = (long)a.g.M * a.g.N;
    hipLaunchKernelGGL(splitk_reduce_px_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, a, p.splits,
                       (int)(MODE == 1 && s.stride == 2 && conv_tap_major(s, 1)));
    MD2_LAUNCH_CHECK();
  }
  return MD2_OK;
}

template <int BM, int BN, int WM, int WN, int KS, int SS, int RR, int CW>
void launch_w_cw(const ConvArgs& a, dim3 grid, hipStream_t st) {
  if constexpr (CW <= BN)
    hipLaunchKernelGGL((conv_wgrad_tap_kernel<BM, BN, 32, WM, WN, KS, KS, SS, RR, CW>), grid,
                       dim3(256), 0, st, a);
}

template <int BM, int BN, int WM, int WN, int KS, int SS, int RR>
int launch_w(int cw, const ConvArgs& a, dim3 grid, hipStream_t st) {
  switch (cw) {
    case 0:
      hipLaunchKernelGGL((conv_wgrad_kernel<BM, BN, 32, WM, WN, KS, KS, SS, RR>), grid, dim3(256), 0,
                         st, a);
      break;
    case 16: launch_w_cw<BM, BN, WM, WN, KS, SS, RR, 16>(a, grid, st); break;
    case 32: launch_w_cw<BM, BN, WM, WN, KS, SS, RR, 32>(a, grid, st); break;
    case 64: launch_w_cw<BM, BN, WM, WN, KS, SS, RR, 64>(a, grid, st); break;
    case 128: launch_w_cw<BM, BN, WM, WN, KS, SS, RR, 128>(a, grid, st); break;
    default: return MD2_ENOTSUP;
  }
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

// stride-2 dgrad output-parity class (cy, cx): input pixels iy = y0 + 2j with (iy + pad) % 2 ==
// cy receive exactly the taps kh % 2 == cy (same for columns)
struct PhaseClass {
  int y0, x0, Hc, Wc, ntaps;
  int taps[16];
};

PhaseClass phase_class(const ConvShape& s, int cy, int cx) {
  PhaseClass c{};
  c.y0 = (cy + s.pad) & 1;
  c.x0 = (cx + s.pad) & 1;
  c.Hc = (s.H - c.y0 + 1) / 2;
  c.Wc = (s.W - c.x0 + 1) / 2;
  static_assert(sizeof(c.taps) / sizeof(c.taps[0]) >= 16, "taps of a 7x7 class");
  for (int kh = cy; kh < s.KH; kh += 2)
    for (int kw = cx; kw < s.KW; kw += 2) c.taps[c.ntaps++] = kh * s.KW + kw;
  return c;
}

}  // namespace

// the k-contiguous kernel (conv_px2.inc) runs every tap-major fwd / dgrad with M > 32 (tiles with
// BM >= 64); MD2_PX_V2=0 selects the previous kernel (A/B)
bool conv_px2_used(const ConvShape& s, int mode) {
  static const int v2 = [] {
    const char* e = getenv("MD2_PX_V2");
    return e ? atoi(e) : 1;
  }();
  if (!v2 || mode > 1 || !conv_tap_major(s, mode)) return false;
  return (mode == 0 ? s.Cout : s.Cin) > 32;
}

bool conv_tap_major(const ConvShape& s, int mode) {
  // MD2_CONV_CHANNEL_MAJOR=<bitmask of modes> forces the channel-major order (debugging)
  static const int forced = [] {
    const char* e = getenv("MD2_CONV_CHANNEL_MAJOR");
    return e ? atoi(e) : 0;
  }();
  if (forced & (1 << mode)) return false;
  switch (mode) {
    case 0: return s.Cin % 16 == 0;                                   // px chunk BK = 16
    case 1: return s.Cout % 16 == 0 && (!s.reflect || (s.H != 3 && s.W != 3));
    default: return s.Cin % 16 == 0;                                  // wgrad CW >= 16
  }
}

// Cout = 1 3x3 convs (disparity heads) run the VALU kernels of head.hip; MD2_HEAD=0 disables
static bool head_path(const ConvShape& s) {
  static const int on = [] {
    const char* e = getenv("MD2_HEAD");
    return e ? atoi(e) : 1;
  }();
  return on && head_conv_ok(s);
}
// tap (c, t) of the packed operand: forward rows m = 0, k = t*Cin + c or c*9 + t; dgrad
// k = co*9 + t = t (Cout = 1, channel-major), row c
static HeadW head_w(const ConvShape& s, int mode, const float* packed) {
  HeadW w{packed, 0, 0};
  if (mode == 0) {
    const long Mpad = round_up(s.Cout, MPAD);
    if (conv_tap_major(s, 0)) { w.sc = Mpad; w.st = (long)s.Cin * Mpad; }
    else { w.sc = 9 * Mpad; w.st = Mpad; }
  } else {
    w.sc = 1;
    w.st = round_up(s.Cin, MPAD);
  }
  return w;
}
static HeadIn head_in(const TensorIn& x) { return HeadIn{x.p0, x.bs0, x.bdiv, x.bhi}; }

size_t conv_fwd_workspace(const ConvShape& s) {
  const long N = (long)s.N * s.Ho * s.Wo;
  const Plan p = plan_px(s.Cout, N, s.Cin * s.KH * s.KW);   // BK does not change the split count

  return p.splits > 1 ? (size_t)p.splits * s.Cout * N * sizeof(float) : 0;
}

size_t conv_dgrad_workspace(const ConvShape& s) {
  if (s.stride == 2 && conv_tap_major(s, 1)) {
    size_t b = 0;
    for (int cls = 0; cls < 4; ++cls) {
      const PhaseClass c = phase_class(s, cls >> 1, cls & 1);
      const long N = (long)s.N * c.Hc * c.Wc;
      const Plan p = plan_px(s.Cin, N, c.ntaps * s.Cout);
      if (p.splits > 1) b = std::max(b, (size_t)p.splits * s.Cin * N * sizeof(float));
    }
    return b;
  }
  const long N = (long)s.N * s.H * s.W;
  const Plan p = plan_px(s.Cin, N, s.Cout * s.KH * s.KW);
  return p.splits > 1 ? (size_t)p.splits * s.Cin * N * sizeof(float) : 0;
}

static size_t wgrad_ws_bytes(const ConvShape& s, int c0) {
  const long K = (long)s.N * s.Ho * s.Wo;
  const long Nc = (long)s.Cin * s.KH * s.KW;
  const WPlan p = plan_wgrad(s, c0);
  const size_t groups = (size_t)std::min(p.splits, WRED_GROUPS);
  return ((size_t)p.splits + groups) * s.Cout * Nc * sizeof(float) +
         (size_t)s.Cout * bias_parts(s.Cout, K) * sizeof(float) + 256;
}

// the split count depends on the concat split only through CW: size for every possible CW
size_t conv_wgrad_workspace(const ConvShape& s) {
  if (head_path(s)) return head_wgrad_workspace(s);
  size_t b = wgrad_ws_bytes(s, s.Cin);
  for (int c0 = 16; c0 <= 128; c0 *= 2) b = std::max(b, wgrad_ws_bytes(s, c0));
  return b;
}

int conv_fwd(const ConvShape& s, const TensorIn& x, const float* wpacked, const TensorOut& y,
             ConvWorkspace ws, hipStream_t st) {
  MD2_TRY(check_shape(s));
  MD2_CHECK_ARG(x.p0 && wpacked && y.p0, "conv_fwd pointers");
  MD2_CHECK_ARG(x.c0 == s.Cin || x.p1 != nullptr, "conv_fwd: second input tensor missing");
  MD2_CHECK_ARG(x.c0 >= s.Cin || !conv_tap_major(s, 0) || x.c0 % 16 == 0,
                "conv_fwd: concat split must be a multiple of 16 channels");
  if (head_path(s) && x.c0 >= s.Cin && y.c0 >= 1) {
    MD2_CHECK_ARG(!conv_px2_used(s, 0), "head: packed layout");
    return head_fwd(s, head_in(x), head_w(s, 0, wpacked), y.bias, y.act, y.p0, y.bs0,
                    y.accumulate, st);
  }
  ConvArgs a{};
  fill_common(a, s);
  a.g.M = s.Cout;
  a.g.N = (long)s.N * s.Ho * s.Wo;
  a.g.K = s.Cin * s.KH * s.KW;
  a.g.Mpad = (int)round_up(s.Cout, MPAD);
  a.fd_pix = make_fastdiv((uint32_t)(s.Ho * s.Wo));
  a.fd_row = make_fastdiv((uint32_t)s.Wo);
  a.fd_bdiv = make_fastdiv((uint32_t)std::min(x.bdiv, 1 << 30));
  a.in = x;
  a.A = wpacked;
  a.out = y;
  a.A_bytes = (uint32_t)(conv_fwd_packed_elems(s) * sizeof(float));
  {
    long ext0 = 0;
    for (int b = 0; b < s.N; ++b)
      ext0 = std::max(ext0, (long)(b % x.bdiv) * x.bs0 + (long)(b / x.bdiv) * x.bhi);
    ext0 += (long)x.c0 * s.H * s.W;
    const long ext1 = x.p1 ? (long)(s.N - 1) * x.bs1 + (long)(s.Cin - x.c0) * s.H * s.W : 0;
    MD2_CHECK_ARG(ext0 * 4 < (long)OOB && ext1 * 4 < (long)OOB, "conv_fwd: tensor exceeds 2 GB");
    a.b0_bytes = (uint32_t)(ext0 * 4);
    a.b1_bytes = (uint32_t)(ext1 * 4);
  }
  const bool bk32 = conv_tap_major(s, 0) && s.Cin % 32 == 0 && (x.c0 >= s.Cin || x.c0 % 32 == 0);
  const Plan p = plan_px(a.g.M, a.g.N, a.g.K, bk32);
  return launch_px<0>(s, a, p, ws, st);
}

int conv_dgrad(const ConvShape& s, const float* dy, const float* wpacked_d, const TensorOut& dx,
               ConvWorkspace ws, hipStream_t st) {
  MD2_TRY(check_shape(s));
  MD2_CHECK_ARG(dy && wpacked_d && dx.p0, "conv_dgrad pointers");
  MD2_CHECK_ARG(!dx.bias && dx.act == ACT_NONE, "conv_dgrad: no bias/activation on dX");
  if (head_path(s) && dx.c0 >= s.Cin) {
    MD2_CHECK_ARG(!conv_px2_used(s, 1) && !conv_tap_major(s, 1), "head: packed layout");
    return head_dgrad(s, dy, head_w(s, 1, wpacked_d), dx.p0, dx.bs0, dx.accumulate, st);
  }
  ConvArgs a{};
  fill_common(a, s);
  a.g.M = s.Cin;
  a.g.N = (long)s.N * s.H * s.W;
  a.g.K = s.Cout * s.KH * s.KW;
  a.g.Mpad = (int)round_up(s.Cin, MPAD);
  a.fd_pix = make_fastdiv((uint32_t)(s.H * s.W));
  a.fd_row = make_fastdiv((uint32_t)s.W);
  a.fd_bdiv = make_fastdiv(1u << 30);
  a.dy = dy;
  a.A = wpacked_d;
  a.out = dx;
  a.A_bytes = (uint32_t)(conv_dgrad_packed_elems(s) * sizeof(float));
  MD2_CHECK_ARG((long)s.N * s.Cout * s.Ho * s.Wo * 4 < (long)OOB, "conv_dgrad: tensor exceeds 2 GB");
  a.b0_bytes = (uint32_t)((long)s.N * s.Cout * s.Ho * s.Wo * 4);
  a.b1_bytes = 0;
  if (s.stride == 2 && conv_tap_major(s, 1)) {
    // four dense GEMMs over the output-parity classes, each with only its own taps
    for (int cls = 0; cls < 4; ++cls) {
      const PhaseClass c = phase_class(s, cls >> 1, cls & 1);
      if (c.Hc <= 0 || c.Wc <= 0 || (c.ntaps == 0 && dx.accumulate)) continue;
      ConvArgs ac = a;
      ac.ph_y0 = c.y0;
      ac.ph_x0 = c.x0;
      for (int t = 0; t < 16; ++t) ac.ph_taps[t] = t < c.ntaps ? c.taps[t] : 0;
      ac.g.N = (long)s.N * c.Hc * c.Wc;
      ac.g.K = c.ntaps * s.Cout;
      ac.fd_pix = make_fastdiv((uint32_t)(c.Hc * c.Wc));
      ac.fd_row = make_fastdiv((uint32_t)c.Wc);
      const Plan p = plan_px(ac.g.M, ac.g.N, ac.g.K, s.Cout % 32 == 0);
      MD2_TRY(launch_px<1>(s, ac, p, ws, st));
    }
    return MD2_OK;
  }
  const Plan p = plan_px(a.g.M, a.g.N, a.g.K, conv_tap_major(s, 1) && s.Cout % 32 == 0);
  return launch_px<1>(s, a, p, ws, st);
}

int conv_wgrad(const ConvShape& s, const TensorIn& x, const float* dy, float* dw, float* db,
               int accumulate, ConvWorkspace ws, hipStream_t st) {
  MD2_TRY(check_shape(s));
  MD2_CHECK_ARG(x.p0 && dy && dw, "conv_wgrad pointers");
  MD2_CHECK_ARG(x.c0 >= s.Cin || x.p1 != nullptr, "conv_wgrad: second input tensor missing");
  if (head_path(s) && x.c0 >= s.Cin)
    return head_wgrad(s, head_in(x), dy, dw, db, accumulate, ws.ptr, ws.bytes, st);
  const WPlan p = plan_wgrad(s, x.c0);
  const bool tap = p.cw > 0;
  ConvArgs a{};
  fill_common(a, s);
  const long Kpix = (long)s.N * s.Ho * s.Wo;
  a.g.M = s.Cout;
  a.g.N = (long)s.Cin * s.KH * s.KW;
  a.g.K = (int)Kpix;
  a.fd_pix = make_fastdiv((uint32_t)(s.Ho * s.Wo));
  a.fd_row = make_fastdiv((uint32_t)s.Wo);
  a.fd_bdiv = make_fastdiv((uint32_t)std::min(x.bdiv, 1 << 30));
  a.in = x;
  a.dy = dy;
  {
    long ext0 = 0;
    for (int b = 0; b < s.N; ++b)
      ext0 = std::max(ext0, (long)(b % x.bdiv) * x.bs0 + (long)(b / x.bdiv) * x.bhi);
    ext0 += (long)std::min(x.c0, s.Cin) * s.H * s.W;
    const long ext1 = x.p1 ? (long)(s.N - 1) * x.bs1 + (long)(s.Cin - x.c0) * s.H * s.W : 0;
    const long extd = (long)s.N * s.Cout * s.Ho * s.Wo;
    MD2_CHECK_ARG(ext0 * 4 < (long)OOB && ext1 * 4 < (long)OOB && extd * 4 < (long)OOB,
                  "conv_wgrad: tensor exceeds 2 GB");
    a.b0_bytes = (uint32_t)(ext0 * 4);
    a.b1_bytes = (uint32_t)(ext1 * 4);
    a.A_bytes = (uint32_t)(extd * 4);
  }
  a.g.kper = p.kper;
  const size_t need = conv_wgrad_workspace(s);
  MD2_CHECK_ARG(ws.ptr && ws.bytes >= need, "conv_wgrad workspace too small");
  a.slab = (float*)ws.ptr;
  const long total = (long)a.g.M * a.g.N;
  const int groups = std::min(p.splits, WRED_GROUPS);
  float* part = a.slab + (long)p.splits * total;
  float* bpart = part + (long)groups * total;
  dim3 grid((unsigned)p.ntiles_n, cdiv(a.g.M, p.BM), p.splits);
  int rc = MD2_ENOTSUP;
#define MD2_W_CASE(KS, SS, RR)                                                                     \
  if (rc == MD2_ENOTSUP && s.KH == KS && s.stride == SS && s.reflect == RR) {                      \
    switch (p.tile) {                                                                              \
      case W32x256: rc = launch_w<32, 256, 1, 4, KS, SS, RR>(p.cw, a, grid, st); break;            \
      case W64x64: rc = launch_w<64, 64, 2, 2, KS, SS, RR>(p.cw, a, grid, st); break;              \
      case W32x128: rc = launch_w<32, 128, 1, 4, KS, SS, RR>(p.cw, a, grid, st); break;            \
      default: rc = launch_w<64, 128, 2, 2, KS, SS, RR>(p.cw, a, grid, st); break;                 \
    }                                                                                              \
  }
  MD2_CONV_COMBOS(MD2_W_CASE)
#undef MD2_W_CASE
  if (rc) {
    set_error("conv_wgrad: unsupported (kernel, stride, padding) combination");
    return rc;
  }
  MD2_LAUNCH_CHECK();
  if (groups > 1) {
    hipLaunchKernelGGL(splitk_reduce_w1_kernel, dim3(cdiv(total, 256), groups), dim3(256), 0, st,
                       a.slab, p.splits, total, groups, part);
    MD2_LAUNCH_CHECK();
    hipLaunchKernelGGL(splitk_reduce_w2_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, part,
                       groups, total, dw, accumulate, (int)a.g.N, tap ? s.Cin : 0, s.KH * s.KW);
  } else {
    hipLaunchKernelGGL(splitk_reduce_w2_kernel, dim3(cdiv(total, 256)), dim3(256), 0, st, a.slab,
                       1, total, dw, accumulate, (int)a.g.N, tap ? s.Cin : 0, s.KH * s.KW);
  }
  MD2_LAUNCH_CHECK();
  if (db) {
    const int parts = bias_parts(s.Cout, Kpix);
    hipLaunchKernelGGL(bias_grad_partial_kernel, dim3(s.Cout, parts), dim3(256), 0, st, dy, s.Cout,
                       (long)s.Ho * s.Wo, Kpix, parts, bpart);
    MD2_LAUNCH_CHECK();
    hipLaunchKernelGGL(bias_grad_final_kernel, dim3(cdiv(s.Cout, 64)), dim3(64), 0, st, bpart,
                       s.Cout, parts, db, accumulate);
    MD2_LAUNCH_CHECK();
  }
  return MD2_OK;
}

int act_backward(const float* out, const float* dout, float* dpre, long n, int act,
                 hipStream_t st) {
  hipLaunchKernelGGL(act_backward_kernel, dim3(cdiv(n, 256)), dim3(256), 0, st, out, dout, dpre, n,
                     act);
  MD2_LAUNCH_CHECK();
  return MD2_OK;
}

}  // namespace md2
