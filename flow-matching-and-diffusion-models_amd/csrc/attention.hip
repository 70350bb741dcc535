// Linear attention (LinearQKVAttention) for the UNet attention blocks (gfx950); the softmax attention runs on
// the MFMA kernels of csrc/attention_mfma.hip.
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
#include <algorithm>
#include <type_traits>

#include "common.h"
#include "../../include/fmdiff.h"

namespace {

// q rows [Tq] and k/v rows [Tk] of one batch.  Self-attention reads all three from one qkv buffer
// [T][3*inner] (cross = 0); SpatialCrossAttention (attention.py:120-189) reads q from the q_proj output
// [Tq][inner] and k | v from the kv_proj output [Tk][2*inner] (cross = 1), with the same raw head split
// (q.reshape(b, heads, Tq, dh), kv.reshape(b, heads, Tk, 2*dh).chunk(2)).  which: 0 q, 1 k, 2 v, 3 output.
struct AGeo {
  int Tq, Tk, heads, dh, inner, raw, cross;
  FMD_HD int parts(int which) const { return which == 3 ? 1 : (cross ? (which ? 2 : 1) : 3); }
  FMD_HD int slot(int which) const { return which == 3 ? 0 : (cross && which ? which - 1 : which); }
  FMD_HD int rows(int which) const { return (which == 1 || which == 2) ? Tk : Tq; }
  // element offset inside one batch's buffer (32-bit: the host checks every buffer < 2^32 elements)
  FMD_DEV unsigned off(int which, int h, int r, int d) const {
    const unsigned P = parts(which), T = rows(which);
    if (raw) {
      const unsigned f = ((unsigned)h * T + r) * P * dh + slot(which) * dh + d;
      const unsigned c = f / T;
      return (f - c * T) * P * inner + c;
    }
    return (unsigned)r * P * inner + slot(which) * inner + h * dh + d;
  }
  FMD_HD size_t qstride() const { return (size_t)Tq * parts(0) * inner; }
  FMD_HD size_t kvstride() const { return (size_t)Tk * parts(1) * inner; }
  FMD_HD size_t ostride() const { return (size_t)Tq * inner; }
  bool fits() const {
    return qstride() < (1ull << 32) && kvstride() < (1ull << 32) && (size_t)Tq * heads * dh < (1ull << 32);
  }
};

// walks consecutive d of one (which, head, row): one division per row instead of one per element
struct ARow {
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
FMD_DEV ARow arow(const AGeo& g, int which, int h, int r, int d0) {
  ARow w;
  w.raw = g.raw;
  w.T = g.rows(which);
  w.ld = g.parts(which) * g.inner;
  if (g.raw) {
    const unsigned f = ((unsigned)h * w.T + r) * g.parts(which) * g.dh + g.slot(which) * g.dh + d0;
    w.c = f / w.T;
    w.t = f - w.c * w.T;
    w.off = 0;
  } else {
    w.t = w.c = 0;
    w.off = g.off(which, h, r, d0);
  }
  return w;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// Linear attention: LinearQKVAttention (src/nn/blocks/attention.py:53-70) inside
// SpatialSelfAttention(use_linear=True) (attention.py:104-117) and SpatialCrossAttention(use_linear=True)
// (attention.py:157-189), same head splits as above (AGeo):
//   ks = softmax_tokens(k), qs = softmax_d(q), A = ks^T v [dh][dh], s = sum_tokens ks [dh],
//   ctx = A / (s + eps), out = qs ctx.
// Token reductions (column softmax statistics, A, s over the Tk key rows; the backward's dctx over the
// Tq query rows) are split over up to LA_MAXCH token chunks per (batch, head) into fp32 partial slabs,
// reduced by a per-(batch, head) kernel -- no atomics, deterministic.  The backward never needs a second
// token pass for the column-softmax Jacobian: sum_n ks*dks = sum_e ctx*dctx + ds*s in closed form.
// state per (batch, head): [ctx D*D | M D | Z D | s D] (fp32, kept from forward for backward).
namespace {

constexpr int LA_D = 64;        // head dims padded to 64 in every LDS tile
constexpr int LA_MAXCH = 64;
constexpr int LA_SB = 64;       // tokens per LDS sub-block
constexpr int LA_STATE = LA_D * LA_D + 3 * LA_D;
constexpr int LA_PART = LA_D * LA_D + LA_D;

struct LaArgs {
  AGeo g;
  int nchq, perq;   // query-row chunks per (batch, head), rows per chunk
  int nchk, perk;   // key-row chunks
  float eps;
};

FMD_DEV void la_range(int T, int per, int c, int& n0, int& n1) {
  n0 = c * per;
  n1 = min(T, n0 + per);
}

// partial column max / sum-exp of k over one key chunk: ws[(bh*nchk + c)][2][D]
__global__ __launch_bounds__(256) void la_kstats(const bf16r* __restrict__ kvsrc, LaArgs a, float* __restrict__ ws) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const AGeo& g = a.g;
  const bf16r* kb = kvsrc + b * g.kvstride();
  const int d = t & 63, gi = t >> 6;
  int n0, n1;
  la_range(g.Tk, a.perk, c, n0, n1);
  float m = -INFINITY, z = 0.f;
  if (d < g.dh) {
    for (int n = n0 + gi; n < n1; n += 4) {
      const float x = bf2f(kb[g.off(1, h, n, d)]);
      const float mn = fmaxf(m, x);
      z = z * __expf(m - mn) + __expf(x - mn);
      m = mn;
    }
  }
  __shared__ float sm[4][64], sz[4][64];
  sm[gi][d] = m;
  sz[gi][d] = z;
  __syncthreads();
  if (t < 64) {
    float M = sm[0][t];
    for (int i = 1; i < 4; ++i) M = fmaxf(M, sm[i][t]);
    float Z = 0.f;
    if (M > -INFINITY)
      for (int i = 0; i < 4; ++i) Z += sz[i][t] * __expf(sm[i][t] - M);
    float* o = ws + ((size_t)(b * g.heads + h) * a.nchk + c) * 2 * LA_D;
    o[t] = M;
    o[LA_D + t] = Z;
  }
}

// combine the chunk statistics of one (batch, head) into M, Z (thread t < 64 = column t)
FMD_DEV void la_combine_stats(int nch, const float* st, float& M, float& Z) {
  const int t = threadIdx.x;
  M = -INFINITY;
  for (int c = 0; c < nch; ++c) M = fmaxf(M, st[(size_t)c * 2 * LA_D + t]);
  Z = 0.f;
  for (int c = 0; c < nch; ++c) {
    const float mc = st[(size_t)c * 2 * LA_D + t];
    if (mc > -INFINITY) Z += st[(size_t)c * 2 * LA_D + LA_D + t] * __expf(mc - M);
  }
}

// stage ks = exp(k - M)/Z and v rows [LA_SB][D] of key rows [n, n + LA_SB) into LDS (zero padded)
FMD_DEV void la_stage_kv(const bf16r* kb, const AGeo& g, int h, int n, int n1, const float* M, const float* Zi,
                         float* ks, float* vs) {
  for (int e = threadIdx.x; e < LA_SB * LA_D; e += blockDim.x) {
    const int j = e >> 6, d = e & 63, r = n + j;
    float kv = 0.f, vv = 0.f;
    if (r < n1 && d < g.dh) {
      kv = __expf(bf2f(kb[g.off(1, h, r, d)]) - M[d]) * Zi[d];
      vv = bf2f(kb[g.off(2, h, r, d)]);
    }
    ks[e] = kv;
    vs[e] = vv;
  }
}

// partial A = ks^T v and s = sum ks over one key chunk: ws_part[(bh*nchk + c)][D*D + D]
__global__ __launch_bounds__(256) void la_ctx_part(const bf16r* __restrict__ kvsrc, LaArgs a,
                                                    const float* __restrict__ wstat, float* __restrict__ state,
                                                    float* __restrict__ part) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const AGeo& g = a.g;
  const int bh = b * g.heads + h;
  const bf16r* kb = kvsrc + b * g.kvstride();
  __shared__ float M[LA_D], Zi[LA_D];
  __shared__ __attribute__((aligned(16))) float ks[LA_SB * LA_D], vs[LA_SB * LA_D];
  if (t < 64) {
    float m, z;
    la_combine_stats(a.nchk, wstat + (size_t)bh * a.nchk * 2 * LA_D, m, z);
    M[t] = m;
    Zi[t] = z > 0.f ? 1.f / z : 0.f;
    if (c == 0) {
      state[(size_t)bh * LA_STATE + LA_D * LA_D + t] = m;
      state[(size_t)bh * LA_STATE + LA_D * LA_D + LA_D + t] = z;
    }
  }
  __syncthreads();
  int n0, n1;
  la_range(g.Tk, a.perk, c, n0, n1);
  const int di = t >> 4, ei = t & 15;
  float acc[4][4] = {};
  float ssum = 0.f;
  for (int n = n0; n < n1; n += LA_SB) {
    la_stage_kv(kb, g, h, n, n1, M, Zi, ks, vs);
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
  float* o = part + ((size_t)bh * a.nchk + c) * LA_PART;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *(float4*)&o[(4 * di + i) * LA_D + 4 * ei] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
  if (t < 64) o[LA_D * LA_D + t] = ssum;
}

// ctx = (sum of partial A) / (sum of partial s + eps), s -> state
__global__ __launch_bounds__(256) void la_ctx_reduce(LaArgs a, const float* __restrict__ part,
                                                      float* __restrict__ state) {
  const int h = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int bh = b * a.g.heads + h;
  const float* p = part + (size_t)bh * a.nchk * LA_PART;
  float* st = state + (size_t)bh * LA_STATE;
  const int d = t >> 2, e0 = (t & 3) * 16;
  float s = 0.f;
  for (int c = 0; c < a.nchk; ++c) s += p[(size_t)c * LA_PART + LA_D * LA_D + d];
  const float inv = 1.f / (s + a.eps);
  for (int e = e0; e < e0 + 16; ++e) {
    float A = 0.f;
    for (int c = 0; c < a.nchk; ++c) A += p[(size_t)c * LA_PART + d * LA_D + e];
    st[d * LA_D + e] = A * inv;
  }
  if ((t & 3) == 0) st[LA_D * LA_D + 2 * LA_D + d] = s;
}

// 4 lanes per query row, 16 dims each: softmax_d(q) of the row -> LDS (fp32, zero padded)
FMD_DEV void la_q_softmax(const bf16r* qb, const AGeo& g, int h, int r, bool live, int d0, float* qv,
                          float* qs_row) {
  float m = -INFINITY;
  ARow w = arow(g, 0, h, live ? r : 0, d0);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    qv[i] = (live && d0 + i < g.dh) ? bf2f(qb[w.cur()]) : -INFINITY;
    w.next();
    m = fmaxf(m, qv[i]);
  }
  m = fmaxf(m, __shfl_xor(m, 1));
  m = fmaxf(m, __shfl_xor(m, 2));
  float z = 0.f;
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    qv[i] = (live && d0 + i < g.dh) ? __expf(qv[i] - m) : 0.f;
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

// out[n][e] = sum_d softmax_d(q[n])[d] * ctx[d][e]; 64 query rows per workgroup, 4 lanes per row
__global__ __launch_bounds__(256) void la_out(const bf16r* __restrict__ qsrc, LaArgs a,
                                              const float* __restrict__ state, bf16r* __restrict__ o) {
  const int h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const AGeo& g = a.g;
  const int bh = b * g.heads + h, dh = g.dh;
  __shared__ __attribute__((aligned(16))) float ctx[LA_D * LA_D], qs[LA_SB * LA_D];
  for (int e = t; e < LA_D * LA_D; e += 256) ctx[e] = state[(size_t)bh * LA_STATE + e];
  const int j = t >> 2, q0 = (t & 3) * 16;
  const int r = blockIdx.x * LA_SB + j;
  const bool live = r < g.Tq;
  float qv[16];
  la_q_softmax(qsrc + b * g.qstride(), g, h, r, live, q0, qv, &qs[j * LA_D]);
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
  bf16r* ob = o + b * g.ostride();
  ARow w = arow(g, 3, h, r, q0);
#pragma unroll
  for (int i = 0; i < 16; ++i) {
    if (q0 + i < dh) ob[w.cur()] = (bf16r)f2bf(acc[i]);
    w.next();
  }
}

// backward, query side, per query chunk: dq (softmax_d Jacobian) and the partial dctx = qs^T dout
__global__ __launch_bounds__(256) void la_bwd_q(const bf16r* __restrict__ qsrc, const bf16r* __restrict__ dout,
                                                LaArgs a, const float* __restrict__ state, float* __restrict__ part,
                                                bf16r* __restrict__ dq_out) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const AGeo& g = a.g;
  const int bh = b * g.heads + h, dh = g.dh;
  const bf16r* qb = qsrc + b * g.qstride();
  const bf16r* dob = dout + b * g.ostride();
  bf16r* dqb = dq_out + b * g.qstride();
  __shared__ __attribute__((aligned(16))) float ctx[LA_D * LA_D], qs[LA_SB * LA_D], dos[LA_SB * LA_D];
  for (int e = t; e < LA_D * LA_D; e += 256) ctx[e] = state[(size_t)bh * LA_STATE + e];
  int n0, n1;
  la_range(g.Tq, a.perq, c, n0, n1);
  const int j = t >> 2, d0 = (t & 3) * 16;   // phase 1: 4 lanes per row, 16 dims each
  const int di = t >> 4, ei = t & 15;       // phase 2: 4x4 tile of dctx
  float acc[4][4] = {};
  for (int n = n0; n < n1; n += LA_SB) {
    __syncthreads();
    for (int e = t; e < LA_SB * LA_D; e += 256) {
      const int jj = e >> 6, dd = e & 63, r = n + jj;
      dos[e] = (r < n1 && dd < dh) ? bf2f(dob[g.off(3, h, r, dd)]) : 0.f;
    }
    const int r = n + j;
    const bool live = r < n1;
    float qv[16];
    la_q_softmax(qb, g, h, r, live, d0, qv, &qs[j * LA_D]);
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
      ARow w = arow(g, 0, h, r, d0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (d0 + i < dh) dqb[w.cur()] = (bf16r)f2bf(qv[i] * (dq[i] - dot));
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
  float* o = part + ((size_t)bh * a.nchq + c) * LA_PART;
#pragma unroll
  for (int i = 0; i < 4; ++i)
    *(float4*)&o[(4 * di + i) * LA_D + 4 * ei] = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
}

// dctx -> dA = dctx/(s+eps), ds = -sum_e dctx*ctx/(s+eps), cc = sum_n ks*dks = sum_e ctx*dctx + ds*s
// into ws_tail[bh][D*D + 2D]
__global__ __launch_bounds__(256) void la_bwd_reduce(LaArgs a, const float* __restrict__ part,
                                                      const float* __restrict__ state, float* __restrict__ tail) {
  const int h = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int bh = b * a.g.heads + h;
  const float* p = part + (size_t)bh * a.nchq * LA_PART;
  const float* st = state + (size_t)bh * LA_STATE;
  float* o = tail + (size_t)bh * (LA_D * LA_D + 2 * LA_D);
  const int d = t >> 2, e0 = (t & 3) * 16;
  const float s = st[LA_D * LA_D + 2 * LA_D + d];
  const float inv = 1.f / (s + a.eps);
  float P = 0.f;
  for (int e = e0; e < e0 + 16; ++e) {
    float gsum = 0.f;
    for (int c = 0; c < a.nchq; ++c) gsum += p[(size_t)c * LA_PART + d * LA_D + e];
    o[d * LA_D + e] = gsum * inv;
    P += gsum * st[d * LA_D + e];
  }
  P += __shfl_xor(P, 1);
  P += __shfl_xor(P, 2);
  if ((t & 3) == 0) {
    const float ds = -P * inv;
    o[LA_D * LA_D + d] = ds;
    o[LA_D * LA_D + LA_D + d] = P + ds * s;
  }
}

// backward, key/value side, per key chunk: dv = ks dA, dk = ks * (v dA^T + ds - cc)
__global__ __launch_bounds__(256) void la_bwd_kv(const bf16r* __restrict__ kvsrc, LaArgs a,
                                                 const float* __restrict__ state, const float* __restrict__ tail,
                                                 bf16r* __restrict__ dkv_out) {
  const int c = blockIdx.x, h = blockIdx.y, b = blockIdx.z, t = threadIdx.x;
  const AGeo& g = a.g;
  const int bh = b * g.heads + h, dh = g.dh;
  const bf16r* kb = kvsrc + b * g.kvstride();
  bf16r* dkb = dkv_out + b * g.kvstride();
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
  la_range(g.Tk, a.perk, c, n0, n1);
  const int j = t >> 2, q0 = (t & 3) * 16;
  for (int n = n0; n < n1; n += LA_SB) {
    la_stage_kv(kb, g, h, n, n1, M, Zi, ks, vs);
    __syncthreads();
    const int r = n + j;
    if (r < n1) {
      float dv[16] = {}, dk[16] = {};
      for (int d = 0; d < LA_D; ++d) {        // dv[e] = sum_d ks[d] dA[d][e]
        const float kd = ks[j * LA_D + d];
#pragma unroll
        for (int i = 0; i < 16; i += 4) {
          const float4 gg = *(const float4*)&dA[d * LA_D + q0 + i];
          dv[i] += kd * gg.x;
          dv[i + 1] += kd * gg.y;
          dv[i + 2] += kd * gg.z;
          dv[i + 3] += kd * gg.w;
        }
      }
#pragma unroll 2
      for (int i = 0; i < 16; ++i) {          // dks[d] = sum_e v[e] dA[d][e]
        float sacc = 0.f;
        for (int e = 0; e < LA_D; e += 4) {
          const float4 gg = *(const float4*)&dA[(q0 + i) * LA_D + e];
          const float4 vv = *(const float4*)&vs[j * LA_D + e];
          sacc += gg.x * vv.x + gg.y * vv.y + gg.z * vv.z + gg.w * vv.w;
        }
        dk[i] = ks[j * LA_D + q0 + i] * (sacc + dsv[q0 + i] - cc[q0 + i]);
      }
      ARow wk = arow(g, 1, h, r, q0), wv = arow(g, 2, h, r, q0);
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        if (q0 + i < dh) {
          dkb[wk.cur()] = (bf16r)f2bf(dk[i]);
          dkb[wv.cur()] = (bf16r)f2bf(dv[i]);
        }
        wk.next();
        wv.next();
      }
    }
    __syncthreads();
  }
}

LaArgs la_args(const AGeo& g, float eps) {
  LaArgs a;
  a.g = g;
  a.nchq = std::min(LA_MAXCH, std::max(1, (g.Tq + 1023) / 1024));
  a.perq = (g.Tq + a.nchq - 1) / a.nchq;
  a.nchk = std::min(LA_MAXCH, std::max(1, (g.Tk + 1023) / 1024));
  a.perk = (g.Tk + a.nchk - 1) / a.nchk;
  a.eps = eps;
  return a;
}

bool geo_ok(const AGeo& g) {
  return g.dh >= 1 && g.dh <= LA_D && g.Tq >= 1 && g.Tk >= 1 && g.heads >= 1 && g.fits();
}

int la_fwd(const bf16r* q, const bf16r* kv, const AGeo& g, int B, float eps, bf16r* o, float* state, float* ws,
           hipStream_t s) {
  const LaArgs a = la_args(g, eps);
  float* part = ws;
  float* wstat = ws + (size_t)B * g.heads * LA_MAXCH * LA_PART;
  const dim3 gk(a.nchk, g.heads, B);
  hipLaunchKernelGGL(la_kstats, gk, dim3(256), 0, s, kv, a, wstat);
  hipLaunchKernelGGL(la_ctx_part, gk, dim3(256), 0, s, kv, a, (const float*)wstat, state, part);
  hipLaunchKernelGGL(la_ctx_reduce, dim3(g.heads, B), dim3(256), 0, s, a, (const float*)part, state);
  hipLaunchKernelGGL(la_out, dim3((g.Tq + LA_SB - 1) / LA_SB, g.heads, B), dim3(256), 0, s, q, a,
                     (const float*)state, o);
  return (int)hipGetLastError();
}

int la_bwd(const bf16r* q, const bf16r* kv, const bf16r* dout, const AGeo& g, int B, float eps, const float* state,
           float* ws, bf16r* dq, bf16r* dkv, hipStream_t s) {
  const LaArgs a = la_args(g, eps);
  float* part = ws;
  float* tail = ws + (size_t)B * g.heads * ((size_t)LA_MAXCH * (LA_PART + 2 * LA_D));
  hipLaunchKernelGGL(la_bwd_q, dim3(a.nchq, g.heads, B), dim3(256), 0, s, q, dout, a, state, part, dq);
  hipLaunchKernelGGL(la_bwd_reduce, dim3(g.heads, B), dim3(256), 0, s, a, (const float*)part, state, tail);
  hipLaunchKernelGGL(la_bwd_kv, dim3(a.nchk, g.heads, B), dim3(256), 0, s, kv, a, state, (const float*)tail, dkv);
  return (int)hipGetLastError();
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
  const AGeo g{T, T, heads, dh, heads * dh, raw, 0};
  if (B < 1 || !geo_ok(g)) return -1;
  return la_fwd((const bf16r*)qkv, (const bf16r*)qkv, g, B, eps, (bf16r*)o, state, ws, (hipStream_t)s);
}

extern "C" int fmd_linear_attention_bwd(const void* qkv, const void* dout, const float* state, float* ws, int32_t B,
                                        int32_t T, int32_t heads, int32_t dh, int32_t raw, float eps, void* dqkv,
                                        fmd_stream_t s) {
  const AGeo g{T, T, heads, dh, heads * dh, raw, 0};
  if (B < 1 || !geo_ok(g)) return -1;
  return la_bwd((const bf16r*)qkv, (const bf16r*)qkv, (const bf16r*)dout, g, B, eps, state, ws, (bf16r*)dqkv,
                (bf16r*)dqkv, (hipStream_t)s);
}

// cross-attention (SpatialCrossAttention): q [B][Tq][inner], kv [B][Tk][2*inner]; linear = LinearQKVAttention
// (state / ws as above), else softmax (lse [B][heads][Tq]; the backward's delta has the same shape)
extern "C" int fmd_cross_attention_fwd(const void* q, const void* kv, int32_t B, int32_t Tq, int32_t Tk,
                                       int32_t heads, int32_t dh, int32_t raw, int32_t linear, float eps, void* o,
                                       float* lse_or_state, float* ws, fmd_stream_t s) {
  const AGeo g{Tq, Tk, heads, dh, heads * dh, raw, 1};
  if (B < 1 || !geo_ok(g)) return -1;
  if (!linear) return -2;   // softmax cross-attention: fmd_attn_mfma_fwd (csrc/attention_mfma.hip)
  return la_fwd((const bf16r*)q, (const bf16r*)kv, g, B, eps, (bf16r*)o, lse_or_state, ws, (hipStream_t)s);
}

extern "C" int fmd_cross_attention_bwd(const void* q, const void* kv, const void* o, const void* dout,
                                       const float* lse_or_state, float* ws_or_delta, int32_t B, int32_t Tq,
                                       int32_t Tk, int32_t heads, int32_t dh, int32_t raw, int32_t linear, float eps,
                                       void* dq, void* dkv, fmd_stream_t s) {
  const AGeo g{Tq, Tk, heads, dh, heads * dh, raw, 1};
  if (B < 1 || !geo_ok(g)) return -1;
  if (!linear) return -2;   // softmax cross-attention: fmd_attn_mfma_bwd (csrc/attention_mfma.hip)
  return la_bwd((const bf16r*)q, (const bf16r*)kv, (const bf16r*)dout, g, B, eps, lse_or_state, ws_or_delta,
                (bf16r*)dq, (bf16r*)dkv, (hipStream_t)s);
}
