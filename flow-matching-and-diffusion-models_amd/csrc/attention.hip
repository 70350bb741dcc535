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
#include <algorithm>
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

// ---------------------------------------------------------------------------------------------
// Linear attention: LinearQKVAttention (src/nn/blocks/attention.py:53-70) inside
// SpatialSelfAttention(use_linear=True) (attention.py:104-117, same raw head split as above):
//   ks = softmax_tokens(k), qs = softmax_d(q), A = ks^T v [dh][dh], s = sum_tokens ks [dh],
//   ctx = A / (s + eps), out = qs ctx.
// Token reductions (column softmax statistics, A, s and the backward's dctx) are split over up to
// LA_MAXCH token chunks per (batch, head) into fp32 partial slabs, reduced by a per-(batch, head)
// kernel -- no atomics, deterministic.  The backward never needs a second token pass for the
// column-softmax Jacobian: sum_n ks*dks = sum_e ctx*dctx + ds*s in closed form.
// state per (batch, head): [ctx D*D | M D | Z D | s D] (fp32, kept from forward for backward).
namespace {

constexpr int LA_D = 64;        // head dims padded to 64 in every LDS tile
constexpr int LA_MAXCH = 64;
constexpr int LA_SB = 64;       // tokens per LDS sub-block
constexpr int LA_STATE = LA_D * LA_D + 3 * LA_D;
constexpr int LA_PART = LA_D * LA_D + LA_D;

struct LaArgs {
  Map mp;
  int nch, per;     // token chunks per (batch, head), tokens per chunk
  float eps;
};

// 32-bit versions of Map::off / Map::ooff (the host checks T * 3 * inner < 2^32)
FMD_DEV unsigned la_off(const Map& mp, int which, int h, int r, int d) {
  if (mp.raw) {
    const unsigned f = (unsigned)h * mp.T * 3 * mp.dh + (unsigned)r * 3 * mp.dh + which * mp.dh + d;
    const unsigned c = f / (unsigned)mp.T;
    return (f - c * mp.T) * 3 * mp.inner + c;
  }
  return (unsigned)r * 3 * mp.inner + which * mp.inner + h * mp.dh + d;
}
FMD_DEV unsigned la_ooff(const Map& mp, int h, int r, int d) {
  if (mp.raw) {
    const unsigned g = (unsigned)h * mp.T * mp.dh + (unsigned)r * mp.dh + d;
    const unsigned c = g / (unsigned)mp.T;
    return (g - c * mp.T) * mp.inner + c;
  }
  return (unsigned)r * mp.inner + h * mp.dh + d;
}

// walks consecutive d of one (which, head, row): one division per row instead of one per element
struct LaRow {
  unsigned t, c, T, ld, off;
  int raw;
  FMD_DEV unsigned cur() const { return raw ? t * ld + c : off; }
  FMD_DEV void next() {
    if (raw) {
      if (++t == T) { t = 0; ++c; }
    } else {
      ++off;
    }
  }
};
FMD_DEV LaRow la_row(const Map& mp, int which, int h, int r, int d0, bool out) {
  LaRow w;
  w.raw = mp.raw;
  w.T = mp.T;
  w.ld = out ? mp.inner : 3 * mp.inner;
  if (mp.raw) {
    const unsigned f = out ? (unsigned)h * mp.T * mp.dh + (unsigned)r * mp.dh + d0
                           : (unsigned)h * mp.T * 3 * mp.dh + (unsigned)r * 3 * mp.dh + which * mp.dh + d0;
    w.c = f / (unsigned)mp.T;
    w.t = f - w.c * mp.T;
    w.off = 0;
  } else {
    w.t = w.c = 0;
    w.off = out ? la_ooff(mp, h, r, d0) : la_off(mp, which, h, r, d0);
  }
  return w;
}

FMD_DEV void la_range(const LaArgs& a, int c, int& n0, int& n1) {
  n0 = c * a.per;
  n1 = min(a.mp.T, n0 + a.per);
}

// partial column max / sum-exp of k over one token chunk: ws[(bh*nch + c)][2][D]
__global__ __launch_bounds__(256) void la_kstats(const bf16r* __restrict__ qkv, LaArgs a, float* __restrict__ ws) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const Map& mp = a.mp;
  const bf16r* base = qkv + (size_t)b * mp.T * 3 * mp.inner;
  const int d = t & 63, g = t >> 6;
  int n0, n1;
  la_range(a, c, n0, n1);
  float m = -INFINITY, z = 0.f;
  if (d < mp.dh) {
    for (int n = n0 + g; n < n1; n += 4) {
      const float x = bf2f(base[la_off(mp, 1, h, n, d)]);
      const float mn = fmaxf(m, x);
      z = z * __expf(m - mn) + __expf(x - mn);
      m = mn;
    }
  }
  __shared__ float sm[4][64], sz[4][64];
  sm[g][d] = m;
  sz[g][d] = z;
  __syncthreads();
  if (t < 64) {
    float M = sm[0][t];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[i][t]);
    float Z = 0.f;
    if (M > -INFINITY)
      for (int i = 0; i < 4; ++i) Z += sz[i][t] * __expf(sm[i][t] - M);
    float* o = ws + ((size_t)(b * mp.heads + h) * a.nch + c) * 2 * LA_D;
    o[t] = M;
    o[LA_D + t] = Z;
  }
}

// combine the chunk statistics of one (batch, head) into M, Z (thread t < 64 = column t)
FMD_DEV void la_combine_stats(const LaArgs& a, const float* st, float& M, float& Z) {
  const int t = threadIdx.x;
  M = -INFINITY;
  for (int c = 0; c < a.nch; ++c) M = fmaxf(M, st[(size_t)c * 2 * LA_D + t]);
  Z = 0.f;
  for (int c = 0; c < a.nch; ++c) {
    const float mc = st[(size_t)c * 2 * LA_D + t];
    if (mc > -INFINITY) Z += st[(size_t)c * 2 * LA_D + LA_D + t] * __expf(mc - M);
  }
}

// stage ks = exp(k - M)/Z and v rows [LA_SB][D] of tokens [n, n + LA_SB) into LDS (zero padded)
FMD_DEV void la_stage_kv(const bf16r* base, const Map& mp, int h, int n, int n1, const float* M, const float* Zi,
                         float* ks, float* vs) {
  for (int e = threadIdx.x; e < LA_SB * LA_D; e += blockDim.x) {
    const int j = e >> 6, d = e & 63, r = n + j;
    float kv = 0.f, vv = 0.f;
    if (r < n1 && d < mp.dh) {
      kv = __expf(bf2f(base[la_off(mp, 1, h, r, d)]) - M[d]) * Zi[d];
      vv = bf2f(base[la_off(mp, 2, h, r, d)]);
    }
    ks[e] = kv;
    if (vs) vs[e] = vv;
  }
}

// partial A = ks^T v and s = sum ks over one token chunk: ws_part[(bh*nch + c)][D*D + D]
__global__ __launch_bounds__(256) void la_ctx_part(const bf16r* __restrict__ qkv, LaArgs a,
                                                    const float* __restrict__ wstat, float* __restrict__ state,
                                                    float* __restrict__ part) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const Map& mp = a.mp;
  const int bh = b * mp.heads + h;
  const bf16r* base = qkv + (size_t)b * mp.T * 3 * mp.inner;
  __shared__ float M[LA_D], Zi[LA_D];
  __shared__ __attribute__((aligned(16))) float ks[LA_SB * LA_D], vs[LA_SB * LA_D];
  if (t < 64) {
    float m, z;
    la_combine_stats(a, wstat + (size_t)bh * a.nch * 2 * LA_D, m, z);
    M[t] = m;
    Zi[t] = z > 0.f ? 1.f / z : 0.f;
    if (c == 0) {
      state[(size_t)bh * LA_STATE + LA_D * LA_D + t] = m;
      state[(size_t)bh * LA_STATE + LA_D * LA_D + LA_D + t] = z;
    }
  }
  __syncthreads();
  int n0, n1;
  la_range(a, c, n0, n1);
  const int di = t >> 4, ei = t & 15;
  float acc[4][4] = {};
  float ssum = 0.f;
  for (int n = n0; n < n1; n += LA_SB) {
    la_stage_kv(base, mp, h, n, n1, M, Zi, ks, vs);
    __syncthreads();
#pragma unroll 4
    for (int j = 0; j < LA_SB; ++j) {
      const float4 kq = *(const float4*)&ks[j * LA_D + 4 * di];
      const float4 vq = *(const float4*)&vs[j * LA_D + 4 * ei];
      const float kk[4] = {kq.x, kq.y, kq.z, kq.w}, vv[4] = {vq.x, vq.y, vq.z, vq.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) acc[i][k2] += kk[i] * vv[k2];
    }
    if (t < 64)
      for (int j = 0; j < LA_SB; ++j) ssum += ks[j * LA_D + t];
    __syncthreads();
  }
  float* o = part + ((size_t)bh * a.nch + c) * LA_PART;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *(float4*)&o[(4 * di + i) * LA_D + 4 * ei] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  if (t < 64) o[LA_D * LA_D + t] = ssum;
}

// ctx = (sum of partial A) / (sum of partial s + eps), s -> state
__global__ __launch_bounds__(256) void la_ctx_reduce(LaArgs a, const float* __restrict__ part,
                                                      float* __restrict__ state) {
  const int h = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int bh = b * a.mp.heads + h;
  const float* p = part + (size_t)bh * a.nch * LA_PART;
  float* st = state + (size_t)bh * LA_STATE;
  const int d = t >> 2, e0 = (t & 3) * 16;
  float s = 0.f;
  for (int c = 0; c < a.nch; ++c) s += p[(size_t)c * LA_PART + LA_D * LA_D + d];
  const float inv = 1.f / (s + a.eps);
  for (int e = e0; e < e0 + 16; ++e) {
    float A = 0.f;
    for (int c = 0; c < a.nch; ++c) A += p[(size_t)c * LA_PART + d * LA_D + e];
    st[d * LA_D + e] = A * inv;
  }
  if ((t & 3) == 0) st[LA_D * LA_D + 2 * LA_D + d] = s;
}

// 4 lanes per token, 16 dims each: softmax_d(q) of the token -> LDS (fp32, zero padded)
FMD_DEV void la_q_softmax(const bf16r* base, const Map& mp, int h, int r, bool live, int d0, float* qv, float* qs_row) {
  float m = -INFINITY;
  LaRow w = la_row(mp, 0, h, live ? r : 0, d0, false);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    qv[i] = (live && d0 + i < mp.dh) ? bf2f(base[w.cur()]) : -INFINITY;
    w.next();
    m = fmaxf(m, qv[i]);
  }
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  float z = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    qv[i] = (live && d0 + i < mp.dh) ? __expf(qv[i] - m) : 0.f;
    z += qv[i];
  }
  z += __shfl_xor(z, 1);
  z += __shfl_xor(z, 2);
  const float zi = live ? 1.f / z : 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    qv[i] *= zi;
    qs_row[d0 + i] = qv[i];
  }
}

// out[n][e] = sum_d softmax_d(q[n])[d] * ctx[d][e]; 64 tokens per workgroup, 4 lanes per token
__global__ __launch_bounds__(256) void la_out(const bf16r* __restrict__ qkv, LaArgs a, const float* __restrict__ state,
                                              bf16r* __restrict__ o) {
  const int h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const Map& mp = a.mp;
  const int bh = b * mp.heads + h, dh = mp.dh;
  __shared__ __attribute__((aligned(16))) float ctx[LA_D * LA_D], qs[LA_SB * LA_D];
  for (int e = t; e < LA_D * LA_D; e += 256) ctx[e] = state[(size_t)bh * LA_STATE + e];
  const int j = t >> 2, q0 = (t & 3) * 16;
  const int r = blockIdx.x * LA_SB + j;
  const bool live = r < mp.T;
  const bf16r* base = qkv + (size_t)b * mp.T * 3 * mp.inner;
  float qv[16];
  la_q_softmax(base, mp, h, r, live, q0, qv, &qs[j * LA_D]);
  __syncthreads();
  if (!live) return;
  float acc[16] = {};
  for (int d = 0; d < LA_D; ++d) {
    const float qd = qs[j * LA_D + d];
#pragma unroll
    for (int i = 0; i < 16; i += 4) {
      const float4 cv = *(const float4*)&ctx[d * LA_D + q0 + i];
      acc[i] += qd * cv.x;
      acc[i + 1] += qd * cv.y;
      acc[i + 2] += qd * cv.z;
      acc[i + 3] += qd * cv.w;
    }
  }
  bf16r* ob = o + (size_t)b * mp.T * mp.inner;
  LaRow w = la_row(mp, 0, h, r, q0, true);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (q0 + i < dh) ob[w.cur()] = (bf16r)f2bf(acc[i]);
    w.next();
  }
}

// backward, query side, per token chunk: dq (softmax_d Jacobian) and the partial dctx = qs^T dout
__global__ __launch_bounds__(256) void la_bwd_q(const bf16r* __restrict__ qkv, const bf16r* __restrict__ dout, LaArgs a,
                                                const float* __restrict__ state, float* __restrict__ part,
                                                bf16r* __restrict__ dqkv) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const Map& mp = a.mp;
  const int bh = b * mp.heads + h, dh = mp.dh;
  const bf16r* base = qkv + (size_t)b * mp.T * 3 * mp.inner;
  const bf16r* dob = dout + (size_t)b * mp.T * mp.inner;
  bf16r* dbase = dqkv + (size_t)b * mp.T * 3 * mp.inner;
  __shared__ __attribute__((aligned(16))) float ctx[LA_D * LA_D], qs[LA_SB * LA_D], dos[LA_SB * LA_D];
  for (int e = t; e < LA_D * LA_D; e += 256) ctx[e] = state[(size_t)bh * LA_STATE + e];
  int n0, n1;
  la_range(a, c, n0, n1);
  const int j = t >> 2, d0 = (t & 3) * 16;   // phase 1: 4 lanes per token, 16 dims each
  const int di = t >> 4, ei = t & 15;       // phase 2: 4x4 tile of dctx
  float acc[4][4] = {};
  for (int n = n0; n < n1; n += LA_SB) {
    __syncthreads();
    for (int e = t; e < LA_SB * LA_D; e += 256) {
      const int jj = e >> 6, dd = e & 63, r = n + jj;
      dos[e] = (r < n1 && dd < dh) ? bf2f(dob[la_ooff(mp, h, r, dd)]) : 0.f;
    }
    const int r = n + j;
    const bool live = r < n1;
    float qv[16];
    la_q_softmax(base, mp, h, r, live, d0, qv, &qs[j * LA_D]);
    __syncthreads();
    // dqs[d] = sum_e dout[e] ctx[d][e]; dq = qs * (dqs - sum_d qs*dqs)
    float dq[16];
    float dot = 0.f;
#pragma unroll
    for (int i = 0; i < 16; ++i) {
      float sacc = 0.f;
      for (int e = 0; e < LA_D; e += 4) {
        const float4 cv = *(const float4*)&ctx[(d0 + i) * LA_D + e];
        const float4 dv = *(const float4*)&dos[j * LA_D + e];
        sacc += cv.x * dv.x + cv.y * dv.y + cv.z * dv.z + cv.w * dv.w;
      }
      dq[i] = sacc;
      dot += qv[i] * sacc;
    }
    dot += __shfl_xor(dot, 1);
    dot += __shfl_xor(dot, 2);
    if (live) {
      LaRow w = la_row(mp, 0, h, r, d0, false);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (d0 + i < dh) dbase[w.cur()] = (bf16r)f2bf(qv[i] * (dq[i] - dot));
        w.next();
      }
    }
#pragma unroll 4
    for (int jj = 0; jj < LA_SB; ++jj) {
      const float4 qq = *(const float4*)&qs[jj * LA_D + 4 * di];
      const float4 dd = *(const float4*)&dos[jj * LA_D + 4 * ei];
      const float q4[4] = {qq.x, qq.y, qq.z, qq.w}, d4[4] = {dd.x, dd.y, dd.z, dd.w};
#pragma unroll
      for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int k2 = 0; k2 < 4; ++k2) acc[i][k2] += q4[i] * d4[k2];
    }
  }
  float* o = part + ((size_t)bh * a.nch + c) * LA_PART;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *(float4*)&o[(4 * di + i) * LA_D + 4 * ei] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
}

// dctx -> dA = dctx/(s+eps), ds = -sum_e dctx*ctx/(s+eps), cc = sum_n ks*dks = sum_e ctx*dctx + ds*s
// into ws_tail[bh][D*D + 2D]
__global__ __launch_bounds__(256) void la_bwd_reduce(LaArgs a, const float* __restrict__ part,
                                                      const float* __restrict__ state, float* __restrict__ tail) {
  const int h = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int bh = b * a.mp.heads + h;
  const float* p = part + (size_t)bh * a.nch * LA_PART;
  const float* st = state + (size_t)bh * LA_STATE;
  float* o = tail + (size_t)bh * (LA_D * LA_D + 2 * LA_D);
  const int d = t >> 2, e0 = (t & 3) * 16;
  const float s = st[LA_D * LA_D + 2 * LA_D + d];
  const float inv = 1.f / (s + a.eps);
  float P = 0.f;
  for (int e = e0; e < e0 + 16; ++e) {
    float g = 0.f;
    for (int c = 0; c < a.nch; ++c) g += p[(size_t)c * LA_PART + d * LA_D + e];
    o[d * LA_D + e] = g * inv;
    P += g * st[d * LA_D + e];
  }
  P += __shfl_xor(P, 1);
  P += __shfl_xor(P, 2);
  if ((t & 3) == 0) {
    const float ds = -P * inv;
    o[LA_D * LA_D + d] = ds;
    o[LA_D * LA_D + LA_D + d] = P + ds * s;
  }
}

// backward, key/value side, per token chunk: dv = ks dA, dk = ks * (v dA^T + ds - cc)
__global__ __launch_bounds__(256) void la_bwd_kv(const bf16r* __restrict__ qkv, LaArgs a,
                                                 const float* __restrict__ state, const float* __restrict__ tail,
                                                 bf16r* __restrict__ dqkv) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const Map& mp = a.mp;
  const int bh = b * mp.heads + h, dh = mp.dh;
  const bf16r* base = qkv + (size_t)b * mp.T * 3 * mp.inner;
  bf16r* dbase = dqkv + (size_t)b * mp.T * 3 * mp.inner;
  __shared__ __attribute__((aligned(16))) float dA[LA_D * LA_D], ks[LA_SB * LA_D], vs[LA_SB * LA_D];
  __shared__ float M[LA_D], Zi[LA_D], dsv[LA_D], cc[LA_D];
  const float* tb = tail + (size_t)bh * (LA_D * LA_D + 2 * LA_D);
  for (int e = t; e < LA_D * LA_D; e += 256) dA[e] = tb[e];
  if (t < 64) {
    const float* st = state + (size_t)bh * LA_STATE + LA_D * LA_D;
    M[t] = st[t];
    Zi[t] = st[LA_D + t] > 0.f ? 1.f / st[LA_D + t] : 0.f;
    dsv[t] = tb[LA_D * LA_D + t];
    cc[t] = tb[LA_D * LA_D + LA_D + t];
  }
  __syncthreads();
  int n0, n1;
  la_range(a, c, n0, n1);
  const int j = t >> 2, q0 = (t & 3) * 16;
  for (int n = n0; n < n1; n += LA_SB) {
    la_stage_kv(base, mp, h, n, n1, M, Zi, ks, vs);
    __syncthreads();
    const int r = n + j;
    if (r < n1) {
      float dv[16] = {}, dk[16] = {};
      for (int d = 0; d < LA_D; ++d) {        // dv[e] = sum_d ks[d] dA[d][e]
        const float kd = ks[j * LA_D + d];
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
          const float4 g = *(const float4*)&dA[d * LA_D + q0 + i];
          dv[i] += kd * g.x;
          dv[i + 1] += kd * g.y;
          dv[i + 2] += kd * g.z;
          dv[i + 3] += kd * g.w;
        }
      }
#pragma unroll 2
      for (int i = 0; i < 16; ++i) {          // dks[d] = sum_e v[e] dA[d][e]
        float sacc = 0.f;
        for (int e = 0; e < LA_D; e += 4) {
          const float4 g = *(const float4*)&dA[(q0 + i) * LA_D + e];
          const float4 vv = *(const float4*)&vs[j * LA_D + e];
          sacc += g.x * vv.x + g.y * vv.y + g.z * vv.z + g.w * vv.w;
        }
        dk[i] = ks[j * LA_D + q0 + i] * (sacc + dsv[q0 + i] - cc[q0 + i]);
      }
      LaRow wk = la_row(mp, 1, h, r, q0, false), wv = la_row(mp, 2, h, r, q0, false);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (q0 + i < dh) {
          dbase[wk.cur()] = (bf16r)f2bf(dk[i]);
          dbase[wv.cur()] = (bf16r)f2bf(dv[i]);
        }
        wk.next();
        wv.next();
      }
    }
    __syncthreads();
  }
}

LaArgs la_args(int32_t T, int32_t heads, int32_t dh, int32_t raw, float eps) {
  LaArgs a;
  a.mp = Map{T, heads, dh, heads * dh, raw};
  a.nch = std::min(LA_MAXCH, std::max(1, (T + 1023) / 1024));
  a.per = (T + a.nch - 1) / a.nch;
  a.eps = eps;
  return a;
}

}  // namespace

// workspace (fp32): [B*heads][LA_MAXCH][LA_PART] partial A/s or dctx | [B*heads][LA_MAXCH][2D] column
// statistics | [B*heads][D*D + 2D] dA, ds, cc
extern "C" size_t fmd_linear_attention_workspace(int32_t B, int32_t heads) {
  return (size_t)B * heads * ((size_t)LA_MAXCH * (LA_PART + 2 * LA_D) + LA_D * LA_D + 2 * LA_D);
}

extern "C" size_t fmd_linear_attention_state(int32_t B, int32_t heads) { return (size_t)B * heads * LA_STATE; }

extern "C" int fmd_linear_attention_fwd(const void* qkv, int32_t B, int32_t T, int32_t heads, int32_t dh, int32_t raw,
                                        float eps, void* o, float* state, float* ws, fmd_stream_t s) {
  if (dh > LA_D || dh < 1 || T < 1 || B < 1 || heads < 1 || (size_t)T * 3 * heads * dh >= (1ull << 32)) return -1;
  const LaArgs a = la_args(T, heads, dh, raw, eps);
  float* part = ws;
  float* wstat = ws + (size_t)B * heads * LA_MAXCH * LA_PART;
  const dim3 gc(a.nch, heads, B);
  hipLaunchKernelGGL(la_kstats, gc, dim3(256), 0, (hipStream_t)s, (const bf16r*)qkv, a, wstat);
  hipLaunchKernelGGL(la_ctx_part, gc, dim3(256), 0, (hipStream_t)s, (const bf16r*)qkv, a, (const float*)wstat, state,
                     part);
  hipLaunchKernelGGL(la_ctx_reduce, dim3(heads, B), dim3(256), 0, (hipStream_t)s, a, (const float*)part, state);
  hipLaunchKernelGGL(la_out, dim3((T + LA_SB - 1) / LA_SB, heads, B), dim3(256), 0, (hipStream_t)s, (const bf16r*)qkv, a,
                     (const float*)state, (bf16r*)o);
  return (int)hipGetLastError();
}

extern "C" int fmd_linear_attention_bwd(const void* qkv, const void* dout, const float* state, float* ws, int32_t B,
                                        int32_t T, int32_t heads, int32_t dh, int32_t raw, float eps, void* dqkv,
                                        fmd_stream_t s) {
  if (dh > LA_D || dh < 1 || T < 1 || B < 1 || heads < 1 || (size_t)T * 3 * heads * dh >= (1ull << 32)) return -1;
  const LaArgs a = la_args(T, heads, dh, raw, eps);
  float* part = ws;
  float* tail = ws + (size_t)B * heads * ((size_t)LA_MAXCH * (LA_PART + 2 * LA_D));
  const dim3 gc(a.nch, heads, B);
  hipLaunchKernelGGL(la_bwd_q, gc, dim3(256), 0, (hipStream_t)s, (const bf16r*)qkv, (const bf16r*)dout, a, state, part,
                     (bf16r*)dqkv);
  hipLaunchKernelGGL(la_bwd_reduce, dim3(heads, B), dim3(256), 0, (hipStream_t)s, a, (const float*)part, state, tail);
  hipLaunchKernelGGL(la_bwd_kv, gc, dim3(256), 0, (hipStream_t)s, (const bf16r*)qkv, a, state, (const float*)tail,
                     (bf16r*)dqkv);
  return (int)hipGetLastError();
}
