// GroupNorm (+ResBlock scale/shift) as folded per-(n,c) affines, forward and
// backward, for gfx950.
//
// Forward: producers emit per-channel partial sums (conv epilogue slab or
// fmd_channel_stats); fmd_gn_prep reduces them per (n, group) in fp64, and
// folds mean/rstd, gamma/beta and the time-embedding scale/shift of
// ResBlockND (src/nn/blocks/residual.py:106-117) into a[n][c], b[n][c] so the
// consuming conv prologue computes silu(a*x + b).
// Backward: with S1 = sum dz, S2 = sum dz*x per (n,c) (conv data-gradient
// epilogue), dx = P*dz + Q*x + R exactly (P, Q, R per (n,c)); gamma/beta and
// scale/shift gradients come from the same sums.
//
// Replaces nn.GroupNorm (src/nn/ops/normalization.py:11-19,
// src/nn/blocks/attention.py:97,210) and its autograd.
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

// x [N][HW][C] bf16 -> slab [N*splits][C][2]; mode 0: (sum x, sum x^2);
// mode 1: (sum dz, sum dz*x) with dz = x, and the second tensor y = the forward input.
__global__ void channel_stats_kernel(const bf16r* __restrict__ x, const bf16r* __restrict__ y0,
                                     const bf16r* __restrict__ y1, int C0, int N, int HW, int C, int rows,
                                     float* __restrict__ out) {
  // block: (n*splits + split, channel block of 64); 256 threads = 8 chunks x 32 pixel lanes
  const int nsplit = HW / rows;
  const int row = blockIdx.x;           // n*nsplit + split
  const int n = row / nsplit, sp = row - n * nsplit;
  const int cblk = blockIdx.y * 64;
  const int t = threadIdx.x;
  const int ch = t & 7, pl = t >> 3;
  const int c = cblk + ch * 8;
  float s1[8], s2[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { s1[e] = 0.f; s2[e] = 0.f; }
  if (c < C) {
    const size_t base = (size_t)n * HW + (size_t)sp * rows;
    for (int p = pl; p < rows; p += 32) {
      const size_t pix = base + p;
      const u32x4 v = *(const u32x4*)(x + pix * C + c);
      float xv[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) { xv[2 * e] = bf_lo(v[e]); xv[2 * e + 1] = bf_hi(v[e]); }
      if (y0) {
        const u32x4 w = (c < C0) ? *(const u32x4*)(y0 + pix * C0 + c) : *(const u32x4*)(y1 + pix * (C - C0) + (c - C0));
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          s1[2 * e] += xv[2 * e];
          s1[2 * e + 1] += xv[2 * e + 1];
          s2[2 * e] += xv[2 * e] * bf_lo(w[e]);
          s2[2 * e + 1] += xv[2 * e + 1] * bf_hi(w[e]);
        }
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) { s1[e] += xv[e]; s2[e] += xv[e] * xv[e]; }
      }
    }
  }
  __shared__ float red[32][8][2][8];
#pragma unroll
  for (int e = 0; e < 8; ++e) { red[pl][ch][0][e] = s1[e]; red[pl][ch][1][e] = s2[e]; }
  __syncthreads();
  if (t < 128) {
    const int cc = t >> 1, k = t & 1;   // 64 channels x 2 sums
    const int chh = cc >> 3, e = cc & 7;
    float a = 0.f;
    for (int i = 0; i < 32; ++i) a += red[i][chh][k][e];
    if (cblk + cc < C) out[((size_t)row * C + cblk + cc) * 2 + k] = a;
  }
}

// Slab fold: out row j = sum of slab rows [j*fold, (j+1)*fold) (C channels x 2 sums each), a block per output
// row reading whole slab rows as coalesced 16-byte vectors, 4 chains per row lane, lanes combined in fixed
// order.  The (n, group) reductions below read a group's Cg channels (16-64 B of each 0.5-4 KiB slab row) from
// every row: on config E's single-sample 128^3 levels (32768 rows of 64 pixels, 32 blocks) that ran at
// < 1 TB/s and 105-293 us per call; folding first leaves them 256 rows.
__global__ __launch_bounds__(256) void stats_fold_kernel(const float* __restrict__ in, int C, int fold,
                                                         float* __restrict__ out) {
  const int V = C / 2;   // 16-byte vectors per slab row
  const size_t r0 = (size_t)blockIdx.x * fold;
  __shared__ f32x4 red[256];
  const int t = threadIdx.x;
  for (int vb = 0; vb < V; vb += 256) {
    const int nv = min(256, V - vb);
    const int R = 256 / nv;   // row lanes
    const int v = t % nv, rl = t / nv;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    if (rl < R) {
      const size_t st = (size_t)R * V;   // f32x4 between a lane's consecutive rows
      const f32x4* p = (const f32x4*)in + (r0 + rl) * V + vb + v;
      int r = rl;
      for (; r + 3 * R < fold; r += 4 * R, p += 4 * st) {
        a0 += p[0];
        a1 += p[st];
        a2 += p[2 * st];
        a3 += p[3 * st];
      }
      for (; r < fold; r += R, p += st) a0 += p[0];
    }
    red[t] = (a0 + a1) + (a2 + a3);
    __syncthreads();
    if (t < nv) {
      f32x4 sum = red[t];
      for (int k = 1; k < R; ++k) sum += red[k * nv + t];
      ((f32x4*)out)[(size_t)blockIdx.x * V + vb + t] = sum;
    }
    __syncthreads();
  }
}

// one block per (n, group)
__global__ void gn_prep_kernel(const float* __restrict__ st0, int rows0, const float* __restrict__ st1, int rows1,
                               int N, int HW, int C0, int C1, int G, float eps, const float* __restrict__ gamma,
                               const float* __restrict__ beta, const float* __restrict__ emb, int emb_stride,
                               int emb_mode, float* __restrict__ a, float* __restrict__ b,
                               float* __restrict__ mr) {
  const int n = blockIdx.x / G, g = blockIdx.x - (blockIdx.x / G) * G;
  const int C = C0 + C1;
  const int Cg = C / G;
  const int c_begin = g * Cg;
  const int E0 = HW / rows0;
  const int E1 = C1 ? HW / rows1 : 0;
  // the affine inputs of this thread's channel, loaded before the slab reduction (their latency under its loads
  // instead of after the block's final barrier)
  float gm = 1.f, bt = 0.f, es = 1.f, esh = 0.f;
  if ((int)threadIdx.x < Cg) {
    const int c = c_begin + threadIdx.x;
    if (gamma) gm = gamma[c];
    if (beta) bt = beta[c];
    if (emb_mode == 1) {
      es = 1.f + emb[(size_t)n * emb_stride + c];
      esh = emb[(size_t)n * emb_stride + C + c];
    }
  }
  double s1 = 0.0, s2 = 0.0;
  const bool in0 = c_begin + Cg <= C0, in1 = c_begin >= C0;
  if ((in0 || in1) && (Cg & 1) == 0) {
    // the group lies in one source: per slab entry its Cg channels are 2*Cg contiguous floats, read as
    // 16-byte vectors; fp32 partials per thread (a few entries), double across threads
    const float* base = in0 ? st0 + (size_t)n * E0 * C0 * 2 + (size_t)c_begin * 2
                            : st1 + (size_t)n * E1 * C1 * 2 + (size_t)(c_begin - C0) * 2;
    const int E = in0 ? E0 : E1;
    const int stride = (in0 ? C0 : C1) * 2;
    // four slab entries per thread in flight (independent partial sums), not one load round trip each
    float f1[4] = {0.f, 0.f, 0.f, 0.f}, f2[4] = {0.f, 0.f, 0.f, 0.f};
    const int step = blockDim.x;
    int e = threadIdx.x;
    for (; e + 3 * step < E; e += 4 * step) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float* p = base + (size_t)(e + u * step) * stride;
        for (int q = 0; q < Cg / 2; ++q) {
          const f32x4 v = *(const f32x4*)(p + 4 * q);
          f1[u] += v[0] + v[2];
          f2[u] += v[1] + v[3];
        }
      }
    }
    for (; e < E; e += step) {
      const float* p = base + (size_t)e * stride;
      for (int q = 0; q < Cg / 2; ++q) {
        const f32x4 v = *(const f32x4*)(p + 4 * q);
        f1[0] += v[0] + v[2];
        f2[0] += v[1] + v[3];
      }
    }
    s1 = (double)((f1[0] + f1[1]) + (f1[2] + f1[3]));
    s2 = (double)((f2[0] + f2[1]) + (f2[2] + f2[3]));
  } else {
    for (int idx = threadIdx.x;; idx += blockDim.x) {
      // enumerate (channel in group, entry)
      const int maxE = E0 > E1 ? E0 : E1;
      if (idx >= Cg * maxE) break;
      const int cl = idx / maxE, e = idx - cl * maxE;
      const int c = c_begin + cl;
      if (c < C0) {
        if (e < E0) {
          const float* p = st0 + (((size_t)n * E0 + e) * C0 + c) * 2;
          s1 += p[0]; s2 += p[1];
        }
      } else {
        if (e < E1) {
          const float* p = st1 + (((size_t)n * E1 + e) * C1 + (c - C0)) * 2;
          s1 += p[0]; s2 += p[1];
        }
      }
    }
  }
  // wave reduction (double), then the waves through LDS
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  __shared__ double r1[16], r2[16];
  if ((threadIdx.x & 63) == 0) { r1[threadIdx.x >> 6] = s1; r2[threadIdx.x >> 6] = s2; }
  __syncthreads();
  if (threadIdx.x == 0) {
    double t1 = 0.0, t2 = 0.0;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) { t1 += r1[w]; t2 += r2[w]; }
    r1[0] = t1;
    r2[0] = t2;
  }
  __syncthreads();
  const double cnt = (double)Cg * HW;
  const double mean = r1[0] / cnt;
  double var = r2[0] / cnt - mean * mean;
  if (var < 0) var = 0;
  const float meanf = (float)mean;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  if (threadIdx.x == 0 && mr) { mr[((size_t)n * G + g) * 2] = meanf; mr[((size_t)n * G + g) * 2 + 1] = rstd; }
  for (int cl = threadIdx.x; cl < Cg; cl += blockDim.x) {   // (channels past the block size: loaded here)
    const int c = c_begin + cl;
    if (cl >= (int)blockDim.x) {
      gm = gamma ? gamma[c] : 1.f;
      bt = beta ? beta[c] : 0.f;
      if (emb_mode == 1) {
        es = 1.f + emb[(size_t)n * emb_stride + c];
        esh = emb[(size_t)n * emb_stride + C + c];
      }
    }
    float av = rstd * gm;
    float bv = bt - meanf * av;
    if (emb_mode == 1) {
      av *= es;
      bv = bv * es + esh;
    }
    a[(size_t)n * C + c] = av;
    b[(size_t)n * C + c] = bv;
  }
}

// one block per (n, group).  T = 256/Cg threads share each channel's slab entries
// (E = HW/rows of them), so the big slabs of the high-resolution levels are
// reduced in parallel; gamma/beta contributions go to a per-(n,c) scratch that
// gn_bwd_gb_kernel folds over n (deterministic, no atomics).
__global__ __launch_bounds__(256) void gn_bwd_prep_kernel(
    const float* __restrict__ s12, int rows, int N, int HW, int C, int G, const float* __restrict__ mr,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ emb, int emb_stride,
    int emb_mode, float* __restrict__ P, float* __restrict__ Q, float* __restrict__ R, float* __restrict__ gb,
    float* __restrict__ demb, int demb_stride, const float* __restrict__ fst, int frows) {
  const int n = blockIdx.x / G, g = blockIdx.x - (blockIdx.x / G) * G;
  const int Cg = C / G;
  const int E = HW / rows;
  const int FE = emb_mode == 2 ? HW / frows : 0;
  __shared__ double sS1[256], sS2[256], sSx[256];
  __shared__ double ch1[256], ch2[256], chx[256];
  __shared__ double red[2][256];
  const int tid = threadIdx.x;
  const int T = 256 / Cg;                 // threads per channel (Cg <= 256)
  const int cl = tid / T, sub = tid - (tid / T) * T;
  double a = 0.0, q = 0.0, sx = 0.0;
  if (cl < Cg) {
    const int c = g * Cg + cl;
    // four slab entries in flight per thread (independent partial sums)
    double a4[4] = {0.0, 0.0, 0.0, 0.0}, q4[4] = {0.0, 0.0, 0.0, 0.0};
    int e = sub;
    for (; e + 3 * T < E; e += 4 * T) {
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const float2 v = *(const float2*)(s12 + (((size_t)n * E + e + u * T) * C + c) * 2);
        a4[u] += v.x;
        q4[u] += v.y;
      }
    }
    for (; e < E; e += T) {
      const float2 v = *(const float2*)(s12 + (((size_t)n * E + e) * C + c) * 2);
      a4[0] += v.x;
      q4[0] += v.y;
    }
    a = (a4[0] + a4[1]) + (a4[2] + a4[3]);
    q = (q4[0] + q4[1]) + (q4[2] + q4[3]);
    for (int e2 = sub; e2 < FE; e2 += T) sx += fst[(((size_t)n * FE + e2) * C + c) * 2];
  }
  sS1[tid] = a; sS2[tid] = q; sSx[tid] = sx;
  __syncthreads();
  if (tid < Cg) {
    double s1 = 0.0, s2 = 0.0, s3 = 0.0;
    for (int k = 0; k < T; ++k) { s1 += sS1[tid * T + k]; s2 += sS2[tid * T + k]; s3 += sSx[tid * T + k]; }
    ch1[tid] = s1; ch2[tid] = s2; chx[tid] = s3;
  }
  __syncthreads();
  const float mean = mr[((size_t)n * G + g) * 2], rstd = mr[((size_t)n * G + g) * 2 + 1];
  double a1 = 0.0, a2 = 0.0;
  if (tid < Cg) {
    const int c = g * Cg + tid;
    const double s = emb_mode == 1 ? 1.0 + (double)emb[(size_t)n * emb_stride + c] : 1.0;
    const double gp = (double)(gamma ? gamma[c] : 1.f) * s;
    a1 = gp * ch1[tid];
    a2 = gp * (double)rstd * (ch2[tid] - (double)mean * ch1[tid]);
  }
  red[0][tid] = a1; red[1][tid] = a2;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if (tid < o) { red[0][tid] += red[0][tid + o]; red[1][tid] += red[1][tid + o]; }
    __syncthreads();
  }
  if (tid < Cg) {
    const double cnt = (double)Cg * HW;
    const double A1 = red[0][0] / cnt, A2 = red[1][0] / cnt;
    const double r = rstd;
    const int c = g * Cg + tid;
    const double s = emb_mode == 1 ? 1.0 + (double)emb[(size_t)n * emb_stride + c] : 1.0;
    const double gm = gamma ? gamma[c] : 1.f;
    const double bt = beta ? beta[c] : 0.f;
    const double gp = gm * s;
    const double S1 = ch1[tid], S2 = ch2[tid];
    const double dzxh = r * (S2 - (double)mean * S1);
    const double Pv = r * gp, Qv = -r * r * A2, Rv = r * r * A2 * mean - r * A1;
    P[(size_t)n * C + c] = (float)Pv;
    Q[(size_t)n * C + c] = (float)Qv;
    R[(size_t)n * C + c] = (float)Rv;
    gb[((size_t)n * C + c) * 2] = (float)(s * dzxh);
    gb[((size_t)n * C + c) * 2 + 1] = (float)(s * S1);
    if (emb_mode == 1 && demb) {
      demb[(size_t)n * demb_stride + c] = (float)(gm * dzxh + bt * S1);
      demb[(size_t)n * demb_stride + C + c] = (float)S1;
    }
    if (emb_mode == 2 && demb)   // sum_hw dx = P*S1 + Q*sum_hw x + R*HW (forward stats give sum_hw x)
      demb[(size_t)n * demb_stride + c] = (float)(Pv * S1 + Qv * chx[tid] + Rv * (double)HW);
  }
}

__global__ void gn_bwd_gb_kernel(const float* __restrict__ gb, int N, int C, float* __restrict__ dgamma,
                                 float* __restrict__ dbeta) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  float a = 0.f, b = 0.f;
  for (int n = 0; n < N; ++n) { a += gb[((size_t)n * C + c) * 2]; b += gb[((size_t)n * C + c) * 2 + 1]; }
  if (dgamma) dgamma[c] += a;
  if (dbeta) dbeta[c] += b;
}

// one block per job: dgamma[c] += sum_n ws[n][c][0], dbeta[c] += sum_n ws[n][c][1] (fixed n order)
struct GbBatch {
  fmd_gb_job j[FMD_GB_MAX];
};
static_assert(sizeof(GbBatch) <= 4096 - 64, "kernel argument segment");

__global__ void gn_gb_fold_kernel(const GbBatch B) {
  const fmd_gb_job J = B.j[blockIdx.x];
  for (int c = threadIdx.x; c < J.C; c += blockDim.x) {
    float a = 0.f, b = 0.f;
    for (int n = 0; n < J.N; ++n) { a += J.ws[((size_t)n * J.C + c) * 2]; b += J.ws[((size_t)n * J.C + c) * 2 + 1]; }
    if (J.dgamma) J.dgamma[c] += a;
    if (J.dbeta) J.dbeta[c] += b;
  }
}

// dx = P*dz + Q*x + R (+ extra), split into two destinations at C0
__global__ void gn_bwd_apply_kernel(const bf16r* __restrict__ dz, const bf16r* __restrict__ x0,
                                    const bf16r* __restrict__ x1, int C0, int C1, long long M, int HW,
                                    const float* __restrict__ P, const float* __restrict__ Q,
                                    const float* __restrict__ R, const bf16r* __restrict__ extra,
                                    bf16r* __restrict__ dx0, int acc0, bf16r* __restrict__ dx1, int acc1) {
  const int C = C0 + C1;
  const int CH = C / 8;
  const long long total = M * CH;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long p = i / CH;
    const int c = (int)(i - p * CH) * 8;
    const int n = (int)(p / HW);
    const u32x4 vz = *(const u32x4*)(dz + p * C + c);
    const bool first = c < C0;
    const u32x4 vx = first ? *(const u32x4*)(x0 + p * C0 + c) : *(const u32x4*)(x1 + p * C1 + (c - C0));
    u32x4 ve = {0u, 0u, 0u, 0u};
    if (extra) ve = *(const u32x4*)(extra + p * C + c);
    const float* pp = P + (size_t)n * C + c;
    const float* qq = Q + (size_t)n * C + c;
    const float* rr = R + (size_t)n * C + c;
    const f32x4 P0 = *(const f32x4*)pp, P1 = *(const f32x4*)(pp + 4);
    const f32x4 Q0 = *(const f32x4*)qq, Q1 = *(const f32x4*)(qq + 4);
    const f32x4 R0 = *(const f32x4*)rr, R1 = *(const f32x4*)(rr + 4);
    const float Pv[8] = {P0[0], P0[1], P0[2], P0[3], P1[0], P1[1], P1[2], P1[3]};
    const float Qv[8] = {Q0[0], Q0[1], Q0[2], Q0[3], Q1[0], Q1[1], Q1[2], Q1[3]};
    const float Rv[8] = {R0[0], R0[1], R0[2], R0[3], R1[0], R1[1], R1[2], R1[3]};
    bf16r* dst = first ? dx0 + p * C0 + c : dx1 + p * C1 + (c - C0);
    const int acc = first ? acc0 : acc1;
    u32x4 old = {0u, 0u, 0u, 0u};
    if (acc) old = *(const u32x4*)dst;
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float lo = Pv[2 * e] * bf_lo(vz[e]) + Qv[2 * e] * bf_lo(vx[e]) + Rv[2 * e];
      float hi = Pv[2 * e + 1] * bf_hi(vz[e]) + Qv[2 * e + 1] * bf_hi(vx[e]) + Rv[2 * e + 1];
      if (extra) { lo += bf_lo(ve[e]); hi += bf_hi(ve[e]); }
      if (acc) { lo += bf_lo(old[e]); hi += bf_hi(old[e]); }
      o[e] = pack2(lo, hi);
    }
    *(u32x4*)dst = o;
  }
}

// t = SiLU(a*x + b) (or the affine alone) over a two-source concat: the GroupNorm(+scale/shift)+SiLU
// prologue materialised once, so every consumer (conv forward, weight gradient) reads it untransformed
__global__ void gn_apply_fwd_kernel(const bf16r* __restrict__ x0, const bf16r* __restrict__ x1, int C0, int C1,
                                    long long M, int HW, const float* __restrict__ a, const float* __restrict__ b,
                                    int silu, bf16r* __restrict__ t) {
  const int C = C0 + C1;
  const int CH = C / 8;
  const long long total = M * CH;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long p = i / CH;
    const int c = (int)(i - p * CH) * 8;
    const int n = (int)(p / HW);
    const u32x4 v = c < C0 ? *(const u32x4*)(x0 + p * C0 + c) : *(const u32x4*)(x1 + p * C1 + (c - C0));
    const float* pa = a + (size_t)n * C + c;
    const float* pb = b + (size_t)n * C + c;
    const f32x4 a0 = *(const f32x4*)pa, a1 = *(const f32x4*)(pa + 4);
    const f32x4 b0 = *(const f32x4*)pb, b1 = *(const f32x4*)(pb + 4);
    const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
    const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float lo = bf_lo(v[e]) * av[2 * e] + bv[2 * e];
      float hi = bf_hi(v[e]) * av[2 * e + 1] + bv[2 * e + 1];
      if (silu) { lo = siluf_(lo); hi = siluf_(hi); }
      o[e] = pack2(lo, hi);
    }
    *(u32x4*)(t + p * C + c) = o;
  }
}

inline int grid_for(long long work, int per_block = 256, int cap = 8192) {
  long long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}

}  // namespace

extern "C" int fmd_channel_stats(const void* x, const void* y0, const void* y1, int32_t C0, int32_t N, int32_t HW,
                                  int32_t C, int32_t rows, float* out, fmd_stream_t stream) {
  if (C % 8 || HW % rows) return -1;
  dim3 grid(N * (HW / rows), (C + 63) / 64);
  hipLaunchKernelGGL(channel_stats_kernel, grid, dim3(256), 0, (hipStream_t)stream, (const bf16r*)x,
                     (const bf16r*)y0, (const bf16r*)y1, C0, N, HW, C, rows, out);
  return (int)hipGetLastError();
}


extern "C" int fmd_stats_fold(const float* slab, int64_t rows_total, int32_t C, int32_t fold, float* out,
                              fmd_stream_t s) {
  if (C < 2 || C % 2 || fold < 1 || rows_total % fold || ((size_t)slab & 15) || ((size_t)out & 15)) return -1;
  if (rows_total / fold > 0x7fffffffLL) return -2;
  hipLaunchKernelGGL(stats_fold_kernel, dim3((unsigned)(rows_total / fold)), dim3(256), 0, (hipStream_t)s, slab, C,
                     fold, out);
  return (int)hipGetLastError();
}

extern "C" int fmd_gn_prep(const float* st0, int32_t rows0, const float* st1, int32_t rows1, int32_t N, int32_t HW,
                           int32_t C0, int32_t C1, int32_t G, float eps, const float* gamma, const float* beta,
                           const float* emb, int32_t emb_stride, int32_t emb_mode, float* a, float* b,
                           float* mean_rstd, fmd_stream_t s) {
  if ((C0 + C1) % G || HW % rows0 || (C1 && HW % rows1)) return -1;
  hipLaunchKernelGGL(gn_prep_kernel, dim3(N * G), dim3(256), 0, (hipStream_t)s, st0, rows0, st1, rows1, N, HW, C0,
                     C1, G, eps, gamma, beta, emb, emb_stride, emb_mode, a, b, mean_rstd);
  return (int)hipGetLastError();
}

extern "C" int fmd_gn_bwd_prep(const float* s12, int32_t rows, int32_t N, int32_t HW, int32_t C, int32_t G,
                               const float* mean_rstd, const float* gamma, const float* beta, const float* emb,
                               int32_t emb_stride, int32_t emb_mode, float* P, float* Q, float* R, float* dgamma,
                               float* dbeta, float* demb, int32_t demb_stride, const float* fwd_st, int32_t fwd_rows,
                               float* ws, fmd_stream_t s) {
  if (C % G || HW % rows || C / G > 256 || !ws) return -1;
  if (emb_mode == 2 && (!fwd_st || HW % fwd_rows)) return -2;
  hipLaunchKernelGGL(gn_bwd_prep_kernel, dim3(N * G), dim3(256), 0, (hipStream_t)s, s12, rows, N, HW, C, G,
                     mean_rstd, gamma, beta, emb, emb_stride, emb_mode, P, Q, R, ws, demb, demb_stride, fwd_st,
                     fwd_rows);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  if (dgamma || dbeta) {
    hipLaunchKernelGGL(gn_bwd_gb_kernel, dim3((C + 255) / 256), dim3(256), 0, (hipStream_t)s, ws, N, C, dgamma,
                       dbeta);
    rc = (int)hipGetLastError();
  }
  return rc;
}

extern "C" int fmd_gn_gb_fold(const fmd_gb_job* jobs, int32_t njobs, fmd_stream_t s) {
  if (njobs < 0 || njobs > FMD_GB_MAX || (njobs && !jobs)) return -1;
  if (njobs == 0) return 0;
  GbBatch B = {};
  for (int i = 0; i < njobs; ++i) {
    if (!jobs[i].ws || jobs[i].N < 1 || jobs[i].C < 1) return -2;
    B.j[i] = jobs[i];
  }
  hipLaunchKernelGGL(gn_gb_fold_kernel, dim3(njobs), dim3(256), 0, (hipStream_t)s, B);
  return (int)hipGetLastError();
}

extern "C" int fmd_gn_bwd_apply(const void* dz, const void* x0, const void* x1, int32_t C0, int32_t C1, int64_t M,
                                int32_t HW, const float* P, const float* Q, const float* R, const void* extra,
                                void* dx0, int32_t acc0, void* dx1, int32_t acc1, fmd_stream_t s) {
  if ((C0 % 8) || (C1 % 8)) return -1;
  const long long work = M * (long long)((C0 + C1) / 8);
  hipLaunchKernelGGL(gn_bwd_apply_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)s, (const bf16r*)dz,
                     (const bf16r*)x0, (const bf16r*)x1, C0, C1, (long long)M, HW, P, Q, R, (const bf16r*)extra,
                     (bf16r*)dx0, acc0, (bf16r*)dx1, acc1);
  return (int)hipGetLastError();
}

// Small levels (HW * C/G <= 16384 elements per group): the whole GroupNorm forward of one
// (n, group) in one workgroup straight from the activation -- statistics (fp32 per thread, fp64 across
// threads, the same E[x^2] - mean^2 form as gn_prep_kernel), the folded a/b (and mean/rstd for the
// backward), and the materialised t = SiLU(a*x + b) over the x0|x1 channel concat.  Replaces
// channel_stats + gn_prep + gn_apply_fwd (three launches) on the generic-conv levels, where each of
// them costs the ~5 us launch floor.  Elements are 4-channel units (8 bytes, C0 % 4 == 0), held in
// registers between the two passes.
namespace {
constexpr int GN_FUSED_UNITS = 16;   // units per thread (256 threads: 4096 units = 16384 elements)
__global__ __launch_bounds__(256) void gn_fused_apply_kernel(
    const bf16r* __restrict__ x0, const bf16r* __restrict__ x1, int C0, int C1, int HW, int G, float eps,
    const float* __restrict__ gamma, const float* __restrict__ beta, const float* __restrict__ emb,
    int emb_stride, int emb_mode, int silu, float* __restrict__ a, float* __restrict__ b,
    float* __restrict__ mr, bf16r* __restrict__ t) {
  const int n = blockIdx.x / G, g = blockIdx.x - (blockIdx.x / G) * G;
  const int C = C0 + C1;
  const int Cg = C / G, Q = Cg / 4;                  // 4-channel units per pixel of the group
  const int U = HW * Q;
  const int tid = threadIdx.x;
  const int cq = tid % Q;                            // 256 % Q == 0: a thread's units share one channel quad
  const int c = g * Cg + cq * 4;
  const bool s0 = c < C0;
  const bf16r* src = s0 ? x0 + c : x1 + (c - C0);
  const int ld = s0 ? C0 : C1;
  const size_t pix0 = (size_t)n * HW;
  // the per-channel parameters are read up front with the activations: one memory round trip, not two
  float gm[4], bt[4], sc[4], sh[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    gm[e] = gamma ? gamma[c + e] : 1.f;
    bt[e] = beta ? beta[c + e] : 0.f;
    sc[e] = emb_mode == 1 ? 1.f + emb[(size_t)n * emb_stride + c + e] : 1.f;
    sh[e] = emb_mode == 1 ? emb[(size_t)n * emb_stride + C + c + e] : 0.f;
  }
  uint2 v[GN_FUSED_UNITS];
  float f1 = 0.f, f2 = 0.f;
#pragma unroll
  for (int k = 0; k < GN_FUSED_UNITS; ++k) {
    const int u = tid + 256 * k;
    v[k] = make_uint2(0u, 0u);
    if (u < U) {
      v[k] = *(const uint2*)(src + (pix0 + u / Q) * ld);
      const float e0 = bf_lo(v[k].x), e1 = bf_hi(v[k].x), e2 = bf_lo(v[k].y), e3 = bf_hi(v[k].y);
      f1 += (e0 + e1) + (e2 + e3);
      f2 += (e0 * e0 + e1 * e1) + (e2 * e2 + e3 * e3);
    }
  }
  double s1 = f1, s2 = f2;
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) {
    s1 += __shfl_xor(s1, o, 64);
    s2 += __shfl_xor(s2, o, 64);
  }
  __shared__ double r1[4], r2[4];
  if ((tid & 63) == 0) { r1[tid >> 6] = s1; r2[tid >> 6] = s2; }
  __syncthreads();
  const double t1 = (r1[0] + r1[1]) + (r1[2] + r1[3]), t2 = (r2[0] + r2[1]) + (r2[2] + r2[3]);
  const double cnt = (double)Cg * HW;
  const double mean = t1 / cnt;
  double var = t2 / cnt - mean * mean;
  if (var < 0) var = 0;
  const float meanf = (float)mean;
  const float rstd = (float)(1.0 / sqrt(var + (double)eps));
  if (tid == 0 && mr) { mr[((size_t)n * G + g) * 2] = meanf; mr[((size_t)n * G + g) * 2 + 1] = rstd; }
  float av[4], bv[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    av[e] = rstd * gm[e];
    bv[e] = bt[e] - meanf * av[e];
    if (emb_mode == 1) {
      av[e] *= sc[e];
      bv[e] = bv[e] * sc[e] + sh[e];
    }
  }
  if (tid < Q) {
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      a[(size_t)n * C + c + e] = av[e];
      b[(size_t)n * C + c + e] = bv[e];
    }
  }
#pragma unroll
  for (int k = 0; k < GN_FUSED_UNITS; ++k) {
    const int u = tid + 256 * k;
    if (u < U) {
      float y0 = bf_lo(v[k].x) * av[0] + bv[0], y1 = bf_hi(v[k].x) * av[1] + bv[1];
      float y2 = bf_lo(v[k].y) * av[2] + bv[2], y3 = bf_hi(v[k].y) * av[3] + bv[3];
      if (silu) { y0 = siluf_(y0); y1 = siluf_(y1); y2 = siluf_(y2); y3 = siluf_(y3); }
      *(uint2*)(t + (pix0 + u / Q) * C + c) = make_uint2(pack2(y0, y1), pack2(y2, y3));
    }
  }
}

}  // namespace

extern "C" int fmd_gn_fused_apply(const void* x0, const void* x1, int32_t C0, int32_t C1, int32_t N, int32_t HW,
                                  int32_t G, float eps, const float* gamma, const float* beta, const float* emb,
                                  int32_t emb_stride, int32_t emb_mode, int32_t silu, float* a, float* b,
                                  float* mean_rstd, void* t, fmd_stream_t s) {
  const int C = C0 + C1;
  if (G < 1 || C % G || (C / G) % 4 || (C0 % 4) || (C1 && !x1) || (emb_mode == 1 && !emb)) return -1;
  const int Q = C / G / 4;
  if (256 % Q || (long long)HW * Q > 256LL * GN_FUSED_UNITS) return -2;
  hipLaunchKernelGGL(gn_fused_apply_kernel, dim3(N * G), dim3(256), 0, (hipStream_t)s, (const bf16r*)x0,
                     (const bf16r*)x1, C0, C1, HW, G, eps, gamma, beta, emb, emb_stride, emb_mode, silu, a, b,
                     mean_rstd, (bf16r*)t);
  return (int)hipGetLastError();
}

extern "C" int fmd_gn_apply_fwd(const void* x0, const void* x1, int32_t C0, int32_t C1, int64_t M, int32_t HW,
                                const float* a, const float* b, int32_t silu, void* t, fmd_stream_t s) {
  if ((C0 % 8) || (C1 % 8) || (C1 && !x1)) return -1;
  const long long work = M * (long long)((C0 + C1) / 8);
  hipLaunchKernelGGL(gn_apply_fwd_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)s, (const bf16r*)x0,
                     (const bf16r*)x1, C0, C1, (long long)M, HW, a, b, silu, (bf16r*)t);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// ResBlockND's out_layers dropout (src/nn/blocks/residual.py:117, nn.Dropout between SiLU and conv2):
// y = x * keep / (1 - p) over the materialised SiLU(GN(h)) operand of conv2, keep = (hash >= p * 2^32) of
// (seed, salt, element index) -- counter-based, so the backward regenerates the forward's mask instead of
// storing it.  seed is read from device memory (a per-forward counter: one hipGraph replay = one fresh
// mask); salt distinguishes the blocks.  With ep_x the same launch is the backward through dropout and the
// SiLU of the GroupNorm prologue: dz = dy * keep / (1 - p) * silu'(a[n][c] * ep_x + b[n][c]).
namespace {

FMD_HD unsigned int fmd_mix32(unsigned int x) {   // "lowbias32" integer finaliser
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

__global__ void dropout_apply_kernel(const bf16r* x, int C, long long M, int HW, unsigned int thr,
                                     float scale, const int* __restrict__ seed, unsigned int salt,
                                     const bf16r* __restrict__ ep_x, const float* __restrict__ a,
                                     const float* __restrict__ b, bf16r* y) {   // y may alias x
  const unsigned int key = fmd_mix32((unsigned int)seed[0] * 0x9e3779b9u + salt);
  const int CH = C / 8;
  const long long total = M * CH;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total; i += (long long)gridDim.x * blockDim.x) {
    const long long p = i / CH;
    const int c = (int)(i - p * CH) * 8;
    const unsigned int e0 = (unsigned int)(p * C + c);     // flat NHWC element index (< 2^32, checked on the host)
    const u32x4 v = *(const u32x4*)(x + p * C + c);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; ++e) m[e] = fmd_mix32(key ^ (e0 + e)) >= thr ? scale : 0.f;
    if (ep_x) {
      const int n = (int)(p / HW);
      const u32x4 h = *(const u32x4*)(ep_x + p * C + c);
      const float* pa = a + (size_t)n * C + c;
      const float* pb = b + (size_t)n * C + c;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        m[2 * e] *= silu_grad(bf_lo(h[e]) * pa[2 * e] + pb[2 * e]);
        m[2 * e + 1] *= silu_grad(bf_hi(h[e]) * pa[2 * e + 1] + pb[2 * e + 1]);
      }
    }
    u32x4 o;
#pragma unroll
    for (int e = 0; e < 4; ++e) o[e] = pack2(bf_lo(v[e]) * m[2 * e], bf_hi(v[e]) * m[2 * e + 1]);
    *(u32x4*)(y + p * C + c) = o;
  }
}

}  // namespace

extern "C" int fmd_dropout_apply(const void* x, int32_t C, int64_t M, int32_t HW, float p, const int32_t* seed,
                                 uint32_t salt, const void* ep_x, const float* ep_a, const float* ep_b, void* y,
                                 fmd_stream_t s) {
  if ((C % 8) || !seed || !(p >= 0.f && p < 1.f) || (ep_x && (!ep_a || !ep_b)) || HW < 1) return -1;
  if (M * (long long)C >= (1LL << 32)) return -2;
  const unsigned int thr = (unsigned int)fmin((double)p * 4294967296.0, 4294967295.0);
  const long long work = M * (long long)(C / 8);
  hipLaunchKernelGGL(dropout_apply_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)s, (const bf16r*)x, C,
                     (long long)M, HW, thr, 1.f / (1.f - p), (const int*)seed, salt, (const bf16r*)ep_x, ep_a, ep_b,
                     (bf16r*)y);
  return (int)hipGetLastError();
}

// ---------------------------------------------------------------------------------------------
// SpatialCrossAttention's context_norm (src/nn/blocks/attention.py:150-151, :177): GroupNorm over the
// flattened context (few channels: the 4-channel VAE latent of configs/LDCT/PixelAttention) straight from
// its fp32 (N, C, Tc) channel-major or (N, Tc, C) token-major layout into the token-major bf16
// [N][Tc][Cpad] operand of the kv 1x1 projection (channels >= C zero); mean / rstd per (sample, group)
// are kept for the gamma / beta gradient.  The context is conditioning data: no gradient flows into it.
namespace {

FMD_DEV float block_sum256(float v, float* red) {
  v = wave_sum(v);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = v;
  __syncthreads();
  return red[0] + red[1] + red[2] + red[3];
}

FMD_DEV float ctx_at(const float* x, size_t base, int C, int T, int tok_major, int c, int r) {
  return tok_major ? x[base + (size_t)r * C + c] : x[base + (size_t)c * T + r];
}

__global__ __launch_bounds__(256) void ctx_norm_fwd_kernel(const float* __restrict__ x, int C, int T, int tok_major,
                                                           int G, float eps, const float* __restrict__ gamma,
                                                           const float* __restrict__ beta, int Cpad,
                                                           bf16r* __restrict__ out, float* __restrict__ mr) {
  const int g = blockIdx.x, n = blockIdx.y, t = threadIdx.x;
  __shared__ float red[4];
  const int Cg = C / G, cnt = Cg * T;
  const size_t base = (size_t)n * C * T;
  float s = 0.f;
  for (int i = t; i < cnt; i += 256) s += ctx_at(x, base, C, T, tok_major, g * Cg + i / T, i % T);
  const float mean = block_sum256(s, red) / cnt;
  float v = 0.f;
  for (int i = t; i < cnt; i += 256) {
    const float d = ctx_at(x, base, C, T, tok_major, g * Cg + i / T, i % T) - mean;
    v += d * d;
  }
  const float rstd = rsqrtf(block_sum256(v, red) / cnt + eps);
  for (int i = t; i < cnt; i += 256) {
    const int c = g * Cg + i / T, r = i % T;
    const float y = (ctx_at(x, base, C, T, tok_major, c, r) - mean) * rstd * gamma[c] + beta[c];
    out[((size_t)n * T + r) * Cpad + c] = (bf16r)f2bf(y);
  }
  if (g == 0)
    for (int i = t; i < (Cpad - C) * T; i += 256) out[((size_t)n * T + i / (Cpad - C)) * Cpad + C + i % (Cpad - C)] = 0;
  if (t == 0) {
    mr[(n * G + g) * 2] = mean;
    mr[(n * G + g) * 2 + 1] = rstd;
  }
}

// dgamma[c] += sum dY * xhat, dbeta[c] += sum dY over all samples and tokens (one workgroup per channel)
__global__ __launch_bounds__(256) void ctx_norm_bwd_kernel(const float* __restrict__ x, int N, int C, int T,
                                                           int tok_major, int G, const float* __restrict__ mr,
                                                           const bf16r* __restrict__ dy, int Cpad,
                                                           float* __restrict__ dgamma, float* __restrict__ dbeta) {
  const int c = blockIdx.x, t = threadIdx.x;
  __shared__ float red[4];
  const int g = c / (C / G);
  float sg = 0.f, sb = 0.f;
  for (long long i = t; i < (long long)N * T; i += 256) {
    const int n = (int)(i / T), r = (int)(i % T);
    const float d = bf2f(dy[((size_t)n * T + r) * Cpad + c]);
    const float xh = (ctx_at(x, (size_t)n * C * T, C, T, tok_major, c, r) - mr[(n * G + g) * 2]) * mr[(n * G + g) * 2 + 1];
    sg += d * xh;
    sb += d;
  }
  sg = block_sum256(sg, red);
  sb = block_sum256(sb, red);
  if (t == 0) {
    dgamma[c] += sg;
    dbeta[c] += sb;
  }
}

}  // namespace

extern "C" int fmd_context_norm_fwd(const float* ctx, int32_t N, int32_t C, int32_t T, int32_t tok_major,
                                    int32_t groups, float eps, const float* gamma, const float* beta, int32_t Cpad,
                                    void* out, float* mr, fmd_stream_t s) {
  if (N < 1 || C < 1 || T < 1 || groups < 1 || C % groups || Cpad < C) return -1;
  hipLaunchKernelGGL(ctx_norm_fwd_kernel, dim3(groups, N), dim3(256), 0, (hipStream_t)s, ctx, C, T, tok_major, groups,
                     eps, gamma, beta, Cpad, (bf16r*)out, mr);
  return (int)hipGetLastError();
}

extern "C" int fmd_context_norm_bwd(const float* ctx, int32_t N, int32_t C, int32_t T, int32_t tok_major,
                                    int32_t groups, const float* mr, const void* dout, int32_t Cpad, float* dgamma,
                                    float* dbeta, fmd_stream_t s) {
  if (N < 1 || C < 1 || T < 1 || groups < 1 || C % groups || Cpad < C) return -1;
  hipLaunchKernelGGL(ctx_norm_bwd_kernel, dim3(C), dim3(256), 0, (hipStream_t)s, ctx, N, C, T, tok_major, groups, mr,
                     (const bf16r*)dout, Cpad, dgamma, dbeta);
  return (int)hipGetLastError();
}
