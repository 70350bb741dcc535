// Token self-attention for the UNet attention blocks (gfx950).
//
// q/k/v come straight out of the fused qkv 1x1-conv (NHWC bf16 [B][T][3*inner]);
// the head split is done by index arithmetic in the loads, so both layouts
// of the reference run without a copy:
//   raw = 1: SpatialSelfAttention's raw reshape (src/nn/blocks/attention.py:111-115):
//            the channel-major (3*inner, T) buffer is reinterpreted as
//            (heads, T, 3*dh): Q[h][r][d] = flat[h*T*3dh + r*3dh + d], K +dh, V +2dh,
//            flat f = c*T + t;  output (heads, T, dh) reinterpreted as (inner, T).
//   raw = 0: DiffusersAttentionND's view/transpose split (attention.py:262-268):
//            Q[h][r][d] = qkv[r][h*dh + d], K at +inner, V at +2*inner.
// Forward: one wave per 64 query rows of one (batch, head), online softmax in
// fp32, K/V staged through LDS in 64-key blocks.  Saves the log-sum-exp so the
// backward recomputes P (flash-style) without storing the T x T scores.
// Replaces F.scaled_dot_product_attention (attention.py:42-44).
#include <type_traits>

#include "common.h"
#include "../../include/fmdiff.h"

namespace {

constexpr int DMAX = 64;

struct Map {
  int T, heads, dh, inner, raw;
  // element offset of (which in {0:q,1:k,2:v}, head, row, d) inside one batch's [T][3*inner] slab
  FMD_DEV long off(int which, int h, int r, int d) const {
    if (raw) {
      const long f = (long)h * T * 3 * dh + (long)r * 3 * dh + which * dh + d;
      const long c = f / T, t = f - (f / T) * T;
      return t * 3 * inner + c;
    }
    return (long)r * 3 * inner + which * inner + h * dh + d;
  }
  // output element (head, row, d) inside one batch's [T][inner] slab
  FMD_DEV long ooff(int h, int r, int d) const {
    if (raw) {
      const long g = (long)h * T * dh + (long)r * dh + d;
      const long c = g / T, t = g - (g / T) * T;
      return t * inner + c;
    }
    return (long)r * inner + h * dh + d;
  }
};

__global__ __launch_bounds__(64) void attn_fwd_kernel(const bf16r* __restrict__ qkv, Map mp, bf16r* __restrict__ o,
                                                      float* __restrict__ lse) {
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int T = mp.T, dh = mp.dh;
  const bf16r* base = qkv + (size_t)b * T * 3 * mp.inner;
  const int r = qblk * 64 + threadIdx.x;
  const bool live = r < T;
  const float scale = 1.0f / sqrtf((float)dh);
  float q[DMAX], acc[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    q[d] = (live && d < dh) ? bf2f(base[mp.off(0, h, r, d)]) * scale : 0.f;
    acc[d] = 0.f;
  }
  __shared__ float ks[64][DMAX + 1], vs[64][DMAX + 1];
  float m = -INFINITY, l = 0.f;
  for (int k0 = 0; k0 < T; k0 += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * dh; i += 64) {
      const int kr = i / dh, d = i - (i / dh) * dh;
      const bool ok = k0 + kr < T;
      ks[kr][d] = ok ? bf2f(base[mp.off(1, h, k0 + kr, d)]) : 0.f;
      vs[kr][d] = ok ? bf2f(base[mp.off(2, h, k0 + kr, d)]) : 0.f;
    }
    __syncthreads();
    const int nk = min(64, T - k0);
    for (int j = 0; j < nk; ++j) {
      float sc = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if (d < dh) sc += q[d] * ks[j][d];
      const float mn = fmaxf(m, sc);
      const float corr = __expf(m - mn);
      const float p = __expf(sc - mn);
      l = l * corr + p;
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if (d < dh) acc[d] = acc[d] * corr + p * vs[j][d];
      m = mn;
    }
  }
  if (!live) return;
  const float inv = 1.f / l;
  bf16r* ob = o + (size_t)b * T * mp.inner;
#pragma unroll
  for (int d = 0; d < DMAX; ++d)
    if (d < dh) ob[mp.ooff(h, r, d)] = (bf16r)f2bf(acc[d] * inv);
  lse[((size_t)b * mp.heads + h) * T + r] = m + logf(l);
}

// pass 1 (per query row): delta = sum_d dO*O, dQ = scale * sum_k dS K
__global__ __launch_bounds__(64) void attn_bwd_q_kernel(const bf16r* __restrict__ qkv, const bf16r* __restrict__ o,
                                                        const bf16r* __restrict__ dout, const float* __restrict__ lse,
                                                        Map mp, float* __restrict__ delta,
                                                        bf16r* __restrict__ dqkv) {
  const int qblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int T = mp.T, dh = mp.dh;
  const bf16r* base = qkv + (size_t)b * T * 3 * mp.inner;
  const bf16r* ob = o + (size_t)b * T * mp.inner;
  const bf16r* dob = dout + (size_t)b * T * mp.inner;
  const int r = qblk * 64 + threadIdx.x;
  const bool live = r < T;
  const float scale = 1.0f / sqrtf((float)dh);
  float q[DMAX], dq[DMAX], dov[DMAX];
  float dl = 0.f;
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    const bool ok = live && d < dh;
    q[d] = ok ? bf2f(base[mp.off(0, h, r, d)]) * scale : 0.f;
    dov[d] = ok ? bf2f(dob[mp.ooff(h, r, d)]) : 0.f;
    dl += ok ? dov[d] * bf2f(ob[mp.ooff(h, r, d)]) : 0.f;
    dq[d] = 0.f;
  }
  const float L = live ? lse[((size_t)b * mp.heads + h) * T + r] : 0.f;
  __shared__ float ks[64][DMAX + 1], vs[64][DMAX + 1];
  for (int k0 = 0; k0 < T; k0 += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * dh; i += 64) {
      const int kr = i / dh, d = i - (i / dh) * dh;
      const bool ok = k0 + kr < T;
      ks[kr][d] = ok ? bf2f(base[mp.off(1, h, k0 + kr, d)]) : 0.f;
      vs[kr][d] = ok ? bf2f(base[mp.off(2, h, k0 + kr, d)]) : 0.f;
    }
    __syncthreads();
    const int nk = min(64, T - k0);
    for (int j = 0; j < nk; ++j) {
      float sc = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if (d < dh) { sc += q[d] * ks[j][d]; dp += dov[d] * vs[j][d]; }
      const float p = __expf(sc - L);
      const float ds = p * (dp - dl);
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if (d < dh) dq[d] += ds * ks[j][d];
    }
  }
  if (!live) return;
  delta[((size_t)b * mp.heads + h) * T + r] = dl;
  bf16r* db = dqkv + (size_t)b * T * 3 * mp.inner;
#pragma unroll
  for (int d = 0; d < DMAX; ++d)
    if (d < dh) db[mp.off(0, h, r, d)] = (bf16r)f2bf(dq[d] * scale);
}

// pass 2 (per key row): dV = sum_q P dO,  dK = scale * sum_q dS Q
__global__ __launch_bounds__(64) void attn_bwd_kv_kernel(const bf16r* __restrict__ qkv, const bf16r* __restrict__ dout,
                                                         const float* __restrict__ lse,
                                                         const float* __restrict__ delta, Map mp,
                                                         bf16r* __restrict__ dqkv) {
  const int kblk = blockIdx.x, h = blockIdx.y, b = blockIdx.z;
  const int T = mp.T, dh = mp.dh;
  const bf16r* base = qkv + (size_t)b * T * 3 * mp.inner;
  const bf16r* dob = dout + (size_t)b * T * mp.inner;
  const int r = kblk * 64 + threadIdx.x;
  const bool live = r < T;
  const float scale = 1.0f / sqrtf((float)dh);
  float kv[DMAX], vv[DMAX], dk[DMAX], dv[DMAX];
#pragma unroll
  for (int d = 0; d < DMAX; ++d) {
    const bool ok = live && d < dh;
    kv[d] = ok ? bf2f(base[mp.off(1, h, r, d)]) : 0.f;
    vv[d] = ok ? bf2f(base[mp.off(2, h, r, d)]) : 0.f;
    dk[d] = 0.f;
    dv[d] = 0.f;
  }
  __shared__ float qs[64][DMAX + 1], dos[64][DMAX + 1], ls[64], dls[64];
  for (int q0 = 0; q0 < T; q0 += 64) {
    __syncthreads();
    for (int i = threadIdx.x; i < 64 * dh; i += 64) {
      const int qr = i / dh, d = i - (i / dh) * dh;
      const bool ok = q0 + qr < T;
      qs[qr][d] = ok ? bf2f(base[mp.off(0, h, q0 + qr, d)]) * scale : 0.f;
      dos[qr][d] = ok ? bf2f(dob[mp.ooff(h, q0 + qr, d)]) : 0.f;
    }
    if (q0 + (int)threadIdx.x < T) {
      ls[threadIdx.x] = lse[((size_t)b * mp.heads + h) * T + q0 + threadIdx.x];
      dls[threadIdx.x] = delta[((size_t)b * mp.heads + h) * T + q0 + threadIdx.x];
    }
    __syncthreads();
    const int nq = min(64, T - q0);
    for (int j = 0; j < nq; ++j) {
      float sc = 0.f, dp = 0.f;
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if (d < dh) { sc += qs[j][d] * kv[d]; dp += dos[j][d] * vv[d]; }
      const float p = __expf(sc - ls[j]);
      const float ds = p * (dp - dls[j]);
#pragma unroll
      for (int d = 0; d < DMAX; ++d)
        if (d < dh) { dv[d] += p * dos[j][d]; dk[d] += ds * qs[j][d]; }
    }
  }
  if (!live) return;
  bf16r* db = dqkv + (size_t)b * T * 3 * mp.inner;
#pragma unroll
  for (int d = 0; d < DMAX; ++d)
    if (d < dh) {
      db[mp.off(1, h, r, d)] = (bf16r)f2bf(dk[d]);   // qs already carries the scale
      db[mp.off(2, h, r, d)] = (bf16r)f2bf(dv[d]);
    }
}


// ---------------------------------------------------------------------------------------------
// Slab kernels (T * dh <= 8192): the (batch, head) Q/K/V are staged ONCE into LDS with coalesced
// 16-byte loads -- the raw-reshape head split is undone during staging by 32-bit index math on the
// head's contiguous channel slice -- then 4 lanes per query (or key) split the head dim, so a
// 256-thread block covers 64 rows and the dot-product chains are dh/4 deep.
// all-reduce over each group of LPR (4 or 16) consecutive lanes with DPP (VALU, no LDS crossbar)
template <int LPR>
FMD_DEV float group_sum(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xf, 0xf, false));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xf, 0xf, false));
  if (LPR == 16) {
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xf, 0xf, false));
    v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x140, 0xf, 0xf, false));
  }
  return v;
}
constexpr int SLAB_MAX = 7936;    // T * dh: two fp32 [T][dh] planes (+ 2T) stay under 64 KiB of LDS

struct Slab {
  int T, dh, inner, raw, h;
  // (t, c_local) of memory element -> (which, row, d); c_local in [0, 3dh) (raw) / which*dh + d (not raw)
  FMD_DEV void split(int t, int cl, int& which, int& r, int& d) const {
    if (raw) {
      const int f = cl * T + t;            // head-local flat index into (T, 3dh)
      r = f / (3 * dh);
      const int rem = f - r * 3 * dh;
      which = rem / dh;
      d = rem - which * dh;
    } else {
      which = cl / dh;
      d = cl - which * dh;
      r = t;
    }
  }
  // memory column (channel) of head-local c_local
  FMD_DEV int col(int cl) const {
    if (raw) return h * 3 * dh + cl;
    const int which = cl / dh;
    return which * inner + h * dh + (cl - which * dh);
  }
  // memory offset (inside one batch's [T][3*inner]) of (which, r, d)
  FMD_DEV int qkv_off(int which, int r, int d) const {
    if (raw) {
      const int f = h * T * 3 * dh + r * 3 * dh + which * dh + d;
      const int c = f / T, t = f - (f / T) * T;
      return t * 3 * inner + c;
    }
    return r * 3 * inner + which * inner + h * dh + d;
  }
  // memory offset (inside one batch's [T][inner]) of output (r, d)
  FMD_DEV int o_off(int r, int d) const {
    if (raw) {
      const int g = h * T * dh + r * dh + d;
      const int c = g / T, t = g - (g / T) * T;
      return t * inner + c;
    }
    return r * inner + h * dh + d;
  }
};

// stage the head's q (scaled), k, v into LDS planes [T][dh] (fp32); a null plane is skipped
FMD_DEV void stage_qkv(const bf16r* base, const Slab& S, float scale, float* qs, float* ks, float* vs) {
  const int W = 3 * S.dh;                 // head-local columns per token (multiple of 8)
  const int nvec = S.T * W / 8;
  for (int e = threadIdx.x; e < nvec; e += blockDim.x) {
    const int t = (e * 8) / W, cl0 = e * 8 - t * W;
    const u32x4 v = *(const u32x4*)(base + (size_t)t * 3 * S.inner + S.col(cl0));   // 8 consecutive columns
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      int which, r, d;
      S.split(t, cl0 + u, which, r, d);
      const float x = (u & 1) ? bf_hi(v[u >> 1]) : bf_lo(v[u >> 1]);
      float* dst = which == 0 ? qs : (which == 1 ? ks : vs);
      if (dst) dst[r * S.dh + d] = which == 0 ? x * scale : x;
    }
  }
}

template <int DG, int LPR>
__global__ __launch_bounds__(256) void attn_fwd_slab(const bf16r* __restrict__ qkv, Slab S, int heads,
                                                     bf16r* __restrict__ o, float* __restrict__ lse) {
  extern __shared__ float sm[];
  const int T = S.T, dh = S.dh;
  float* ks = sm;
  float* vs = ks + T * dh;
  const int b = blockIdx.z;
  S.h = blockIdx.y;
  const bf16r* base = qkv + (size_t)b * T * 3 * S.inner;
  const float scale = 1.0f / sqrtf((float)dh);
  stage_qkv(base, S, scale, nullptr, ks, vs);
  __syncthreads();
  const int r = blockIdx.x * (256 / LPR) + (int)(threadIdx.x / LPR), g = threadIdx.x & (LPR - 1);
  const bool live = r < T;
  const int d0 = g * DG;
  float q[DG], acc[DG];
#pragma unroll
  for (int i = 0; i < DG; ++i) {
    q[i] = (live && d0 + i < dh) ? bf2f(base[S.qkv_off(0, r, d0 + i)]) * scale : 0.f;
    acc[i] = 0.f;
  }
  float m = -INFINITY, l = 0.f;
  for (int j = 0; j < T; ++j) {
    float sc = 0.f;
#pragma unroll
    for (int i = 0; i < DG; ++i)
      if (d0 + i < dh) sc += q[i] * ks[j * dh + d0 + i];
    sc = group_sum<LPR>(sc);
    const float mn = fmaxf(m, sc);
    const float corr = __expf(m - mn);
    const float p = __expf(sc - mn);
    l = l * corr + p;
#pragma unroll
    for (int i = 0; i < DG; ++i)
      if (d0 + i < dh) acc[i] = acc[i] * corr + p * vs[j * dh + d0 + i];
    m = mn;
  }
  if (!live) return;
  const float inv = 1.f / l;
  bf16r* ob = o + (size_t)b * T * S.inner;
#pragma unroll
  for (int i = 0; i < DG; ++i)
    if (d0 + i < dh) ob[S.o_off(r, d0 + i)] = (bf16r)f2bf(acc[i] * inv);
  if (g == 0) lse[((size_t)b * heads + S.h) * T + r] = m + logf(l);
}

// dQ per query row: delta = dO.O, dS = P (dO.V - delta), dQ = scale * sum_k dS K
template <int DG, int LPR>
__global__ __launch_bounds__(256) void attn_bwd_q_slab(const bf16r* __restrict__ qkv, const bf16r* __restrict__ o,
                                                       const bf16r* __restrict__ dout, const float* __restrict__ lse,
                                                       Slab S, int heads, float* __restrict__ delta,
                                                       bf16r* __restrict__ dqkv) {
  extern __shared__ float sm[];
  const int T = S.T, dh = S.dh;
  float* ks = sm;
  float* vs = ks + T * dh;
  const int b = blockIdx.z;
  S.h = blockIdx.y;
  const bf16r* base = qkv + (size_t)b * T * 3 * S.inner;
  const float scale = 1.0f / sqrtf((float)dh);
  stage_qkv(base, S, scale, nullptr, ks, vs);
  __syncthreads();
  const int r = blockIdx.x * (256 / LPR) + (int)(threadIdx.x / LPR), g = threadIdx.x & (LPR - 1);
  const bool live = r < T;
  const int d0 = g * DG;
  const bf16r* ob = o + (size_t)b * T * S.inner;
  const bf16r* dob = dout + (size_t)b * T * S.inner;
  float q[DG], dov[DG], dq[DG];
  float dl = 0.f;
#pragma unroll
  for (int i = 0; i < DG; ++i) {
    const bool ok = live && d0 + i < dh;
    q[i] = ok ? bf2f(base[S.qkv_off(0, r, d0 + i)]) * scale : 0.f;
    dov[i] = ok ? bf2f(dob[S.o_off(r, d0 + i)]) : 0.f;
    dl += ok ? dov[i] * bf2f(ob[S.o_off(r, d0 + i)]) : 0.f;
    dq[i] = 0.f;
  }
  dl = group_sum<LPR>(dl);
  const float L = live ? lse[((size_t)b * heads + S.h) * T + r] : 0.f;
  for (int j = 0; j < T; ++j) {
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int i = 0; i < DG; ++i)
      if (d0 + i < dh) { sc += q[i] * ks[j * dh + d0 + i]; dp += dov[i] * vs[j * dh + d0 + i]; }
    sc = group_sum<LPR>(sc);
    dp = group_sum<LPR>(dp);
    const float ds = __expf(sc - L) * (dp - dl);
#pragma unroll
    for (int i = 0; i < DG; ++i)
      if (d0 + i < dh) dq[i] += ds * ks[j * dh + d0 + i];
  }
  if (!live) return;
  if (g == 0) delta[((size_t)b * heads + S.h) * T + r] = dl;
  bf16r* db = dqkv + (size_t)b * T * 3 * S.inner;
#pragma unroll
  for (int i = 0; i < DG; ++i)
    if (d0 + i < dh) db[S.qkv_off(0, r, d0 + i)] = (bf16r)f2bf(dq[i] * scale);
}

// dK, dV per key row: dV = sum_q P dO, dK = sum_q dS (scale Q)
template <int DG, int LPR>
__global__ __launch_bounds__(256) void attn_bwd_kv_slab(const bf16r* __restrict__ qkv, const bf16r* __restrict__ dout,
                                                        const float* __restrict__ lse,
                                                        const float* __restrict__ delta, Slab S, int heads,
                                                        bf16r* __restrict__ dqkv) {
  extern __shared__ float sm[];
  const int T = S.T, dh = S.dh;
  float* qs = sm;
  float* dos = qs + T * dh;
  float* ls = dos + T * dh;
  float* dls = ls + T;
  const int b = blockIdx.z;
  S.h = blockIdx.y;
  const bf16r* base = qkv + (size_t)b * T * 3 * S.inner;
  const bf16r* dob = dout + (size_t)b * T * S.inner;
  stage_qkv(base, S, 1.0f / sqrtf((float)dh), qs, nullptr, nullptr);
  for (int e = threadIdx.x; e < T * dh; e += blockDim.x) {
    const int rr = e / dh, d = e - rr * dh;
    dos[e] = bf2f(dob[S.o_off(rr, d)]);
  }
  for (int e = threadIdx.x; e < T; e += blockDim.x) {
    ls[e] = lse[((size_t)b * heads + S.h) * T + e];
    dls[e] = delta[((size_t)b * heads + S.h) * T + e];
  }
  __syncthreads();
  const int r = blockIdx.x * (256 / LPR) + (int)(threadIdx.x / LPR), g = threadIdx.x & (LPR - 1);
  const bool live = r < T;
  const int d0 = g * DG;
  float kv[DG], vv[DG], dk[DG], dv[DG];
#pragma unroll
  for (int i = 0; i < DG; ++i) {
    const bool ok = live && d0 + i < dh;
    kv[i] = ok ? bf2f(base[S.qkv_off(1, r, d0 + i)]) : 0.f;
    vv[i] = ok ? bf2f(base[S.qkv_off(2, r, d0 + i)]) : 0.f;
    dk[i] = dv[i] = 0.f;
  }
  for (int j = 0; j < T; ++j) {
    float sc = 0.f, dp = 0.f;
#pragma unroll
    for (int i = 0; i < DG; ++i)
      if (d0 + i < dh) { sc += qs[j * dh + d0 + i] * kv[i]; dp += dos[j * dh + d0 + i] * vv[i]; }
    sc = group_sum<LPR>(sc);
    dp = group_sum<LPR>(dp);
    const float p = __expf(sc - ls[j]);
    const float ds = p * (dp - dls[j]);
#pragma unroll
    for (int i = 0; i < DG; ++i)
      if (d0 + i < dh) { dv[i] += p * dos[j * dh + d0 + i]; dk[i] += ds * qs[j * dh + d0 + i]; }
  }
  if (!live) return;
  bf16r* db = dqkv + (size_t)b * T * 3 * S.inner;
#pragma unroll
  for (int i = 0; i < DG; ++i)
    if (d0 + i < dh) {
      db[S.qkv_off(1, r, d0 + i)] = (bf16r)f2bf(dk[i]);
      db[S.qkv_off(2, r, d0 + i)] = (bf16r)f2bf(dv[i]);
    }
}

// (DG, LPR): head-dim elements per lane and lanes per row; 16 lanes per row once dh >= 32, so a
// T = 64 head needs 4 blocks and a 8-image batch with 4 heads fills 128 blocks
template <typename F>
int dispatch_dg(int dh, F&& f) {
  if (dh <= 8) return f(std::integral_constant<int, 2>{}, std::integral_constant<int, 4>{});
  if (dh <= 16) return f(std::integral_constant<int, 4>{}, std::integral_constant<int, 4>{});
  if (dh <= 32) return f(std::integral_constant<int, 2>{}, std::integral_constant<int, 16>{});
  return f(std::integral_constant<int, 4>{}, std::integral_constant<int, 16>{});
}

}  // namespace

extern "C" int fmd_attention_fwd(const void* qkv, int32_t B, int32_t T, int32_t heads, int32_t dh, int32_t raw,
                                 void* o, float* lse, fmd_stream_t s) {
  if (dh > DMAX || dh < 1) return -1;
  if (T * dh <= SLAB_MAX && dh % 8 == 0) {
    Slab S{T, dh, heads * dh, raw, 0};
    const size_t shm = (size_t)2 * T * dh * 4;
    return dispatch_dg(dh, [&](auto dg, auto lpr) {
      constexpr int LPR = decltype(lpr)::value;
      const dim3 grid((T + 256 / LPR - 1) / (256 / LPR), heads, B);
      hipLaunchKernelGGL((attn_fwd_slab<decltype(dg)::value, LPR>), grid, dim3(256), shm, (hipStream_t)s,
                         (const bf16r*)qkv, S, heads, (bf16r*)o, lse);
      return (int)hipGetLastError();
    });
  }
  Map mp{T, heads, dh, heads * dh, raw};
  dim3 grid((T + 63) / 64, heads, B);
  hipLaunchKernelGGL(attn_fwd_kernel, grid, dim3(64), 0, (hipStream_t)s, (const bf16r*)qkv, mp, (bf16r*)o, lse);
  return (int)hipGetLastError();
}

extern "C" int fmd_attention_bwd(const void* qkv, const void* o, const void* dout, const float* lse, float* delta,
                                  int32_t B, int32_t T, int32_t heads, int32_t dh, int32_t raw, void* dqkv,
                                  fmd_stream_t s) {
  if (dh > DMAX || dh < 1) return -1;
  if (T * dh <= SLAB_MAX && dh % 8 == 0) {
    Slab S{T, dh, heads * dh, raw, 0};
    return dispatch_dg(dh, [&](auto dg, auto lpr) {
      constexpr int DG = decltype(dg)::value, LPR = decltype(lpr)::value;
      const dim3 grid((T + 256 / LPR - 1) / (256 / LPR), heads, B);
      hipLaunchKernelGGL((attn_bwd_q_slab<DG, LPR>), grid, dim3(256), (size_t)2 * T * dh * 4, (hipStream_t)s,
                         (const bf16r*)qkv, (const bf16r*)o, (const bf16r*)dout, lse, S, heads, delta, (bf16r*)dqkv);
      int rc = (int)hipGetLastError();
      if (rc) return rc;
      hipLaunchKernelGGL((attn_bwd_kv_slab<DG, LPR>), grid, dim3(256), (size_t)(2 * T * dh + 2 * T) * 4,
                         (hipStream_t)s, (const bf16r*)qkv, (const bf16r*)dout, lse, delta, S, heads,
                         (bf16r*)dqkv);
      return (int)hipGetLastError();
    });
  }
  Map mp{T, heads, dh, heads * dh, raw};
  dim3 grid((T + 63) / 64, heads, B);
  hipLaunchKernelGGL(attn_bwd_q_kernel, grid, dim3(64), 0, (hipStream_t)s, (const bf16r*)qkv, (const bf16r*)o,
                     (const bf16r*)dout, lse, mp, delta, (bf16r*)dqkv);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  hipLaunchKernelGGL(attn_bwd_kv_kernel, grid, dim3(64), 0, (hipStream_t)s, (const bf16r*)qkv, (const bf16r*)dout, lse,
                     delta, mp, (bf16r*)dqkv);
  return (int)hipGetLastError();
}
