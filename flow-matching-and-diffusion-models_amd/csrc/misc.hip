// Small wavefront kernels around the UNet hot path (gfx950): weight layout
// preparation, NCHW<->NHWC staging, sinusoidal timestep features and the
// time-embedding / ResBlock emb_layers linears, the FM / DDPM train-step
// input preparation and MSE loss, the FlowMatchEuler / DDPM / DDIM step
// updates, and a flat fused AdamW.
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

inline int grid_for(long long work, int per_block = 256, int cap = 16384) {
  long long b = (work + per_block - 1) / per_block;
  if (b > cap) b = cap;
  if (b < 1) b = 1;
  return (int)b;
}
#define GRID_STRIDE(i, total) \
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < (total); i += (long long)gridDim.x * blockDim.x)

// mode 0: forward  out[k][tap][c] (rows k >= K and channels c >= C zero; Kpad x T x Cpad)
// mode 1: data-grad out[c][tap][k] (Cpad rows, Kpad inner)
// mode 2: data-grad of nearest-x2 upsample + 3x3 conv: 4x4 effective taps, out[c][16][k]
// T: taps of the kernel (ks*ks in 2-D, ks^3 in 3-D); ks is read by mode 2 only (2-D up-dgrad)
__global__ void prep_weights_kernel(const float* __restrict__ w, int K, int C, int ks, int T, int mode, int Kpad,
                                    int Cpad, bf16r* __restrict__ out) {
  if (mode == 0) {
    const long long total = (long long)Kpad * T * Cpad;
    GRID_STRIDE(i, total) {
      const int c = (int)(i % Cpad);
      const long long r = i / Cpad;
      const int tap = (int)(r % T);
      const int k = (int)(r / T);
      float v = (k < K && c < C) ? w[((size_t)k * C + c) * T + tap] : 0.f;
      out[i] = (bf16r)f2bf(v);
    }
  } else if (mode == 1 || mode == 3) {
    // mode 3: taps flipped (T-1-tap) -> the data gradient of a stride-1 conv as a forward gather
    const long long total = (long long)Cpad * T * Kpad;
    GRID_STRIDE(i, total) {
      const int k = (int)(i % Kpad);
      const long long r = i / Kpad;
      const int tap = (int)(r % T);
      const int c = (int)(r / T);
      const int st = mode == 3 ? T - 1 - tap : tap;
      float v = (k < K && c < C) ? w[((size_t)k * C + c) * T + st] : 0.f;
      out[i] = (bf16r)f2bf(v);
    }
  } else {
    // 1-D effective taps over dY rows 2i-1 .. 2i+2:  r0: W2, r1: W1+W2, r2: W0+W1, r3: W0
    const long long total = (long long)Cpad * 16 * Kpad;
    GRID_STRIDE(i, total) {
      const int k = (int)(i % Kpad);
      const long long r = i / Kpad;
      const int tap = (int)(r % 16);
      const int c = (int)(r / 16);
      const int ry = tap >> 2, rx = tap & 3;
      float v = 0.f;
      if (k < K && c < C) {
        const int ylo = (ry == 0) ? 2 : (ry == 1 ? 1 : 0), yhi = (ry == 3) ? 0 : (ry == 2 ? 1 : 2);
        const int xlo = (rx == 0) ? 2 : (rx == 1 ? 1 : 0), xhi = (rx == 3) ? 0 : (rx == 2 ? 1 : 2);
        for (int ky = ylo; ky <= yhi; ++ky)
          for (int kx = xlo; kx <= xhi; ++kx) v += w[((size_t)k * C + c) * 9 + ky * 3 + kx];
      }
      out[i] = (bf16r)f2bf(v);
    }
  }
}

__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int HW, int Cpad, bf16r* __restrict__ y) {
  const long long total = (long long)N * HW * Cpad;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % Cpad);
    const long long p = i / Cpad;
    const int n = (int)(p / HW), hw = (int)(p % HW);
    y[i] = (bf16r)f2bf(c < C ? x[((size_t)n * C + c) * HW + hw] : 0.f);
  }
}

__global__ void nhwc_to_nchw_kernel(const void* __restrict__ y, int src_f32, int N, int C, int HW, int Cs,
                                    float* __restrict__ x) {
  const long long total = (long long)N * C * HW;
  GRID_STRIDE(i, total) {
    const int hw = (int)(i % HW);
    const long long r = i / HW;
    const int c = (int)(r % C), n = (int)(r / C);
    const size_t src = ((size_t)n * HW + hw) * Cs + c;
    x[i] = src_f32 ? ((const float*)y)[src] : bf2f(((const bf16r*)y)[src]);
  }
}

// timestep_embedding (src/nn/ops/time_embedding.py:4-32), fp32 like the reference
// t_scale / t_trunc: the FM trainer's integer timesteps (t * (N-1)).long() (flow_matching_lib.py:153)
__global__ void temb_kernel(const float* __restrict__ t, int N, int dim, int flip, int shift, float neg_log_period,
                            float t_scale, int t_trunc, float* __restrict__ out) {
  const int half = dim / 2;
  const long long total = (long long)N * dim;
  GRID_STRIDE(i, total) {
    const int j = (int)(i % dim), n = (int)(i / dim);
    float v = 0.f;
    if (j < 2 * half) {
      int jj = j;
      if (flip) jj = (j < half) ? j + half : j - half;   // [cos, sin]
      const int f = jj < half ? jj : jj - half;
      const float e = (neg_log_period * (float)f) / (float)max(half - shift, 1);
      float tv = t[n] * t_scale;
      if (t_trunc) tv = (float)(long long)tv;
      const float arg = tv * expf(e);
      v = jj < half ? sinf(arg) : cosf(arg);
    }
    out[i] = v;
  }
}

// y[b][o] = sum_i f(x[b][i]) w[o][i] + bias[o]; one wave per output row, B <= BM.  Rows b >= B read row B - 1 (so
// the unrolled loads carry no branch and issue together) and are never stored.  The first form guarded every x load
// with b < B, which serialised them: ~20 us for the 512 x 128 time-MLP layer.
template <int BM>
__global__ __launch_bounds__(256) void linear_kernel(const float* __restrict__ x, int B, int I,
                                                     const float* __restrict__ w, const float* __restrict__ bias,
                                                     int O, int in_silu, float* __restrict__ y, int ys) {
  const int wid = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
  const int lane = threadIdx.x & 63;
  if (wid >= O) return;
  float acc[BM];
#pragma unroll
  for (int b = 0; b < BM; ++b) acc[b] = 0.f;
#pragma unroll 2
  for (int i = lane; i < I; i += 64) {
    const float wv = w[(size_t)wid * I + i];
    float xv[BM];
#pragma unroll
    for (int b = 0; b < BM; ++b) xv[b] = x[(size_t)min(b, B - 1) * I + i];
#pragma unroll
    for (int b = 0; b < BM; ++b) acc[b] += wv * (in_silu ? siluf_(xv[b]) : xv[b]);
  }
#pragma unroll
  for (int b = 0; b < BM; ++b) {
    if (b < B) {
      const float s = wave_sum(acc[b]);
      if (lane == 0) y[(size_t)b * ys + wid] = s + (bias ? bias[wid] : 0.f);
    }
  }
}

// dw[o][i] += sum_b dy[b][o] f(x[b][i]);  db[o] += sum_b dy[b][o]
__global__ void linear_dw_kernel(const float* __restrict__ x, int B, int I, int O, int in_silu,
                                 const float* __restrict__ dy, int dys, float* __restrict__ dw,
                                 float* __restrict__ db) {
  const long long total = (long long)O * I;
  GRID_STRIDE(idx, total) {
    const int i = (int)(idx % I), o = (int)(idx / I);
    float s = 0.f;
    for (int b = 0; b < B; ++b) {
      float xv = x[(size_t)b * I + i];
      if (in_silu) xv = siluf_(xv);
      s += dy[(size_t)b * dys + o] * xv;
    }
    dw[idx] += s;
    if (db && i == 0) {
      float t = 0.f;
      for (int b = 0; b < B; ++b) t += dy[(size_t)b * dys + o];
      db[o] += t;
    }
  }
}

// dx[b][i] (+)= f'(x) * sum_o dy[b][o] w[o][i].  Grid (I/64, B): a block owns 64 columns of one batch row; its 4 waves
// sum contiguous quarters of the O rows (dy row in LDS, w rows read coalesced, 8 in flight), then meet in LDS in
// fixed order -- deterministic, no atomics, no memset.  (The first form, grid (I/64, O/256) with fp32 atomics across
// the O blocks, ran the time MLP's 512 x 512 layer on 16 blocks: 75 us per train step.)
__global__ __launch_bounds__(256) void linear_dx_kernel(const float* __restrict__ x, int B, int I,
                                                        const float* __restrict__ w, int O, int in_silu,
                                                        const float* __restrict__ dy, int dys,
                                                        float* __restrict__ dx, int acc) {
  extern __shared__ float dyr[];   // [O] this block's dy row
  __shared__ float red[4][64];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int i = blockIdx.x * 64 + lane, b = blockIdx.y;
  for (int o = threadIdx.x; o < O; o += 256) dyr[o] = dy[(size_t)b * dys + o];
  __syncthreads();
  const int per = (O + 3) / 4, o0 = wv * per, o1 = min(O, o0 + per);
  float a0 = 0.f, a1 = 0.f;
  if (i < I) {
    int o = o0;
    for (; o + 8 <= o1; o += 8) {
      float wv8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) wv8[k] = w[(size_t)(o + k) * I + i];
#pragma unroll
      for (int k = 0; k < 8; k += 2) {
        a0 += dyr[o + k] * wv8[k];
        a1 += dyr[o + k + 1] * wv8[k + 1];
      }
    }
    for (; o < o1; ++o) a0 += dyr[o] * w[(size_t)o * I + i];
  }
  red[wv][lane] = a0 + a1;
  __syncthreads();
  if (wv == 0 && i < I) {
    float sv = (red[0][lane] + red[1][lane]) + (red[2][lane] + red[3][lane]);
    if (in_silu) sv *= silu_grad(x[(size_t)b * I + i]);
    float* d = dx + (size_t)b * I + i;
    *d = acc ? *d + sv : sv;
  }
}

__global__ void silu_bwd_kernel(const float* __restrict__ x, const float* __restrict__ dy, float* __restrict__ dx,
                                long long n) {
  GRID_STRIDE(i, n) dx[i] = dy[i] * silu_grad(x[i]);
}

// model input: ch [0,Cx) = ca[n]*x0 + cb[n]*noise (or noise if ca == NULL), [Cx,Cx+Cc) = cond, rest 0
__global__ void noise_prepare_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                     const float* __restrict__ ca, const float* __restrict__ cb,
                                     const float* __restrict__ cond, int N, int HW, int Cx, int Cc, int Cpad,
                                     bf16r* __restrict__ inp) {
  const long long total = (long long)N * HW * Cpad;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % Cpad);
    const long long p = i / Cpad;
    const int n = (int)(p / HW), hw = (int)(p % HW);
    float v = 0.f;
    if (c < Cx) {
      const size_t s = ((size_t)n * Cx + c) * HW + hw;
      v = ca ? (cb ? ca[n] * x0[s] + cb[n] * noise[s] : (1.0f - ca[n]) * x0[s] + ca[n] * noise[s]) : noise[s];
    } else if (c < Cx + Cc) {
      v = cond[((size_t)n * Cc + (c - Cx)) * HW + hw];
    }
    inp[i] = (bf16r)f2bf(v);
  }
}

// diffusers DDPMScheduler.add_noise in fp32: out = sa[t[n]] * x0 + sb[t[n]] * noise with both products
// rounded before the add (no FMA contraction), which is torch's eager operation order: bit-exact.
__global__ void add_noise_kernel(const float* __restrict__ x0, const float* __restrict__ noise,
                                 const float* __restrict__ sa, const float* __restrict__ sb,
                                 const long long* __restrict__ ts, long long per, int N, float* __restrict__ out) {
  const long long total = (long long)N * per;
  GRID_STRIDE(i, total) {
#pragma clang fp contract(off)
    const long long t = ts[i / per];
    const float a = sa[t] * x0[i];
    const float b = sb[t] * noise[i];
    out[i] = a + b;
  }
}

// partial sums of (pred - target)^2; dpred = scale * 2 (pred - target) / numel (bf16, NHWC, Kpad channels)
__global__ void mse_kernel(const float* __restrict__ pred, int Kpad, const float* __restrict__ ta,
                           const float* __restrict__ tb, float tb_sign, int N, int Cx, int HW, float inv_numel,
                           float grad_scale, float* __restrict__ partial, bf16r* __restrict__ dpred) {
  const long long total = (long long)N * HW * Kpad;
  float s = 0.f;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % Kpad);
    const long long p = i / Kpad;
    float g = 0.f;
    if (c < Cx) {
      const int n = (int)(p / HW), hw = (int)(p % HW);
      const size_t ti = ((size_t)n * Cx + c) * HW + hw;
      float target = ta[ti];
      if (tb) target = target + tb_sign * tb[ti];
      const float dlt = pred[i] - target;
      s += dlt * dlt;
      g = grad_scale * 2.f * dlt * inv_numel;
    }
    if (dpred) dpred[i] = (bf16r)f2bf(g);
  }
  __shared__ float red[256];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) partial[blockIdx.x] = red[0];
}

__global__ void sum_partials_kernel(const float* __restrict__ partial, int n, float scale, float* __restrict__ out) {
  __shared__ double red[256];
  double s = 0.0;
  for (int i = threadIdx.x; i < n; i += 256) s += partial[i];
  red[threadIdx.x] = s;
  __syncthreads();
  for (int o = 128; o > 0; o >>= 1) {
    if ((int)threadIdx.x < o) red[threadIdx.x] += red[threadIdx.x + o];
    __syncthreads();
  }
  if (threadIdx.x == 0) out[0] = (float)(red[0] * scale);
}

// torch.optim.AdamW (foreach=False arithmetic), flat fp32 buffers
__global__ void adamw_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                             float* __restrict__ v, long long n, float lr, float b1, float b2, float eps, float wd,
                             float bc1, float bc2_sqrt) {
  GRID_STRIDE(i, n) {
    float pv = p[i];
    const float gv = g[i];
    pv = pv * (1.f - lr * wd);
    float mv = m[i];
    mv = mv + (gv - mv) * (1.f - b1);
    float vv = v[i] * b2 + (1.f - b2) * gv * gv;
    m[i] = mv;
    v[i] = vv;
    const float denom = sqrtf(vv) / bc2_sqrt + eps;
    pv = pv - (lr / bc1) * (mv / denom);
    p[i] = pv;
  }
}

// Same update with the step count read from device memory and the LR of
// get_cosine_schedule_with_warmup (flow_matching_lib.py:76-79) computed on device,
// so a captured train-step graph replays with the right schedule.
__global__ void adamw_sched_kernel(float* __restrict__ p, const float* __restrict__ g, float* __restrict__ m,
                                   float* __restrict__ v, long long n, const int* __restrict__ step_ctr,
                                   float base_lr, int warmup, int total, float b1, float b2, float eps, float wd,
                                   float grad_scale, int vec) {
  const int step = step_ctr[0] + 1;          // optimizer.step() count, 1-based
  const int s = step - 1;                    // lr_scheduler.step() calls so far
  double lam;
  if (s < warmup) {
    lam = (double)s / (double)(warmup > 1 ? warmup : 1);
  } else {
    const double prog = (double)(s - warmup) / (double)((total - warmup) > 1 ? (total - warmup) : 1);
    lam = 0.5 * (1.0 + cos(3.14159265358979323846 * 2.0 * 0.5 * prog));
    if (lam < 0) lam = 0;
  }
  const float lr = (float)(base_lr * lam);
  const float bc1 = (float)(1.0 - pow((double)b1, step));
  const float bc2s = sqrtf((float)(1.0 - pow((double)b2, step)));
  auto upd = [&](float& pv, float gv, float& mv, float& vv) {
    gv *= grad_scale;
    pv = pv * (1.f - lr * wd);
    mv = mv + (gv - mv) * (1.f - b1);
    vv = vv * b2 + (1.f - b2) * gv * gv;
    const float denom = sqrtf(vv) / bc2s + eps;
    pv = pv - (lr / bc1) * (mv / denom);
  };
  // 16-byte accesses over the (16-byte aligned) flat buffers; the n % 4 tail element-wise
  const long long n4 = vec ? n >> 2 : 0;
  GRID_STRIDE(i, n4) {
    f32x4 pv = ((const f32x4*)p)[i], gv = ((const f32x4*)g)[i], mv = ((const f32x4*)m)[i], vv = ((const f32x4*)v)[i];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      float pe = pv[e], me = mv[e], ve = vv[e];
      upd(pe, gv[e], me, ve);
      pv[e] = pe;
      mv[e] = me;
      vv[e] = ve;
    }
    ((f32x4*)p)[i] = pv;
    ((f32x4*)m)[i] = mv;
    ((f32x4*)v)[i] = vv;
  }
  for (long long i = 4 * n4 + (long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (long long)gridDim.x * blockDim.x) {
    float pv = p[i], mv = m[i], vv = v[i];
    upd(pv, g[i], mv, vv);
    p[i] = pv;
    m[i] = mv;
    v[i] = vv;
  }
}

// FlowMatchEuler: x += (sigma[i+1] - sigma[i]) * v   (fp32), then write the next model input
__global__ void flow_euler_kernel(float* __restrict__ x, const float* __restrict__ vout, int Kpad,
                                  const float* __restrict__ sigmas, const int* __restrict__ index, int N, int Cx,
                                  int HW, const float* __restrict__ cond, int Cc, int Cpad, bf16r* __restrict__ next) {
#pragma clang fp contract(off)
  const int idx = index[0];
  const float ds = sigmas[idx + 1] - sigmas[idx];
  const long long total = (long long)N * HW;
  GRID_STRIDE(p, total) {
    const int n = (int)(p / HW), hw = (int)(p % HW);
    for (int c = 0; c < Cx; ++c) {
      const size_t xi = ((size_t)n * Cx + c) * HW + hw;
      const float nv = x[xi] + ds * vout[p * Kpad + c];   // eager order (no FMA): bit-exact
      x[xi] = nv;
      if (next) next[p * Cpad + c] = (bf16r)f2bf(nv);
    }
    if (next) {
      for (int c = 0; c < Cc; ++c) next[p * Cpad + Cx + c] = (bf16r)f2bf(cond[((size_t)n * Cc + c) * HW + hw]);
      for (int c = Cx + Cc; c < Cpad; ++c) next[p * Cpad + c] = 0;
    }
  }
}

// DDPM / DDIM (eps-prediction): coef table row idx = [sqrt_b, sqrt_a, c_x0, c_xt, std, clip, c_eps]
//   x0 = clip((x - sqrt_b*eps)/sqrt_a);  prev = c_x0*x0 + c_xt*x + c_eps*eps + std*z
__global__ void ddpm_step_kernel(float* __restrict__ x, const float* __restrict__ eps, int Kpad,
                                 const float* __restrict__ coef, const int* __restrict__ index,
                                 const float* __restrict__ noise, int noise_base, int N, int Cx, int HW,
                                 const float* __restrict__ cond, int Cc, int Cpad, bf16r* __restrict__ next) {
#pragma clang fp contract(off)
  const int idx = index[0];
  // variance-noise row: noise_base >= 0 -> a per-step table whose row 0 is step noise_base; < 0 -> one buffer
  const size_t nrow = noise_base >= 0 ? (size_t)(idx - noise_base) : 0;
  const float* cf = coef + idx * 7;
  const float sqrt_b = cf[0], sqrt_a = cf[1], cx0 = cf[2], cxt = cf[3], sd = cf[4], clip = cf[5], ceps = cf[6];
  const long long total = (long long)N * HW;
  GRID_STRIDE(p, total) {
    const int n = (int)(p / HW), hw = (int)(p % HW);
    for (int c = 0; c < Cx; ++c) {
      const size_t xi = ((size_t)n * Cx + c) * HW + hw;
      const float e = eps[p * Kpad + c];
      const float xv = x[xi];
      // every product / sum rounded on its own (no FMA contraction, correctly rounded division): diffusers'
      // eager operation order, so the step is bit-exact with the fp32 torch expression
      float x0 = (xv - sqrt_b * e) / sqrt_a;
      if (clip > 0.f) x0 = fminf(fmaxf(x0, -clip), clip);
      float pv = cxt != 0.f ? cx0 * x0 + cxt * xv : cx0 * x0;
      if (ceps != 0.f) pv = pv + ceps * e;
      if (noise && sd > 0.f) pv = pv + sd * noise[nrow * N * Cx * HW + xi];
      x[xi] = pv;
      if (next) next[p * Cpad + c] = (bf16r)f2bf(pv);
    }
    if (next) {
      for (int c = 0; c < Cc; ++c) next[p * Cpad + Cx + c] = (bf16r)f2bf(cond[((size_t)n * Cc + c) * HW + hw]);
      for (int c = Cx + Cc; c < Cpad; ++c) next[p * Cpad + c] = 0;
    }
  }
}

__global__ void fill_from_table_kernel(const float* __restrict__ table, const int* __restrict__ index, float* out,
                                       int N) {
  const int i = threadIdx.x;
  if (i < N) out[i] = table[index[0]];
}

// out[0:n] = table[index[0]*n : index[0]*n + n]  (one row of a per-step table, chosen on the device)
__global__ void gather_row_kernel(const float* __restrict__ table, const int* __restrict__ index, long long n,
                                  float* __restrict__ out) {
  const float* src = table + (long long)index[0] * n;
  GRID_STRIDE(i, n) out[i] = src[i];
}

// out = sum_k c[k] * in[k] over n fp32 elements (k < nin <= FMD_LINCOMB_MAX): the multistep solver
// updates (DPM-Solver++, UniPC) with their per-step scalar coefficients folded on the host
__global__ void lincomb_kernel(const fmd_lincomb_desc D) {
  const long long n4 = D.n / 4;
  const bool vec = (D.n & 3) == 0;
  if (vec) {
    GRID_STRIDE(i, n4) {
      f32x4 acc = {0.f, 0.f, 0.f, 0.f};
      for (int k = 0; k < D.nin; ++k) {
        const f32x4 v = ((const f32x4*)D.in[k])[i];
#pragma unroll
        for (int e = 0; e < 4; ++e) acc[e] = __builtin_fmaf(D.c[k], v[e], acc[e]);
      }
      ((f32x4*)D.out)[i] = acc;
    }
  } else {
    GRID_STRIDE(i, D.n) {
      float acc = 0.f;
      for (int k = 0; k < D.nin; ++k) acc = __builtin_fmaf(D.c[k], D.in[k][i], acc);
      D.out[i] = acc;
    }
  }
}

// fmd_sched_step (include/fmdiff.h): one DPM-Solver / UniPC step, coefficients from the device-indexed table
__global__ void sched_step_kernel(const fmd_sched_step_desc D) {
  const int i = D.index[0];
  const float* c = D.coef + (size_t)i * FMD_SCHED_NCOEF;
  float* const rw = D.ring[i & 3];
  const float* const r1 = D.ring[(i - 1) & 3];
  const float* const r2 = D.ring[(i - 2) & 3];
  const float* const r3 = D.ring[(i - 3) & 3];
  const bool corr = c[2] != 0.f;
  const long long total = (long long)D.N * D.HW;
  GRID_STRIDE(p, total) {
    const int n = (int)(p / D.HW), hw = (int)(p % D.HW);
    for (int ch = 0; ch < D.Cx; ++ch) {
      const size_t xi = ((size_t)n * D.Cx + ch) * D.HW + hw;
      const float xv = D.x[xi];
      float m = 0.f;
      m = __builtin_fmaf(c[0], xv, m);
      m = __builtin_fmaf(c[1], D.eps[p * D.Kpad + ch], m);
      rw[xi] = m;
      float xc = xv;
      if (corr) {
        float a = 0.f;
        a = __builtin_fmaf(c[3], D.last[xi], a);
        a = __builtin_fmaf(c[4], r1[xi], a);
        a = __builtin_fmaf(c[5], r2[xi], a);
        a = __builtin_fmaf(c[6], r3[xi], a);
        a = __builtin_fmaf(c[7], m, a);
        xc = a;
      }
      if (D.last) D.last[xi] = xc;
      float pv = 0.f;
      pv = __builtin_fmaf(c[8], xc, pv);
      pv = __builtin_fmaf(c[9], m, pv);
      pv = __builtin_fmaf(c[10], r1[xi], pv);
      pv = __builtin_fmaf(c[11], r2[xi], pv);
      D.x[xi] = pv;
      if (D.next) ((bf16r*)D.next)[p * D.Cpad + ch] = (bf16r)f2bf(pv);
    }
    if (D.next) {
      bf16r* nx = (bf16r*)D.next;
      for (int ch = 0; ch < D.Cc; ++ch) nx[p * D.Cpad + D.Cx + ch] = (bf16r)f2bf(D.cond[((size_t)n * D.Cc + ch) * D.HW + hw]);
      for (int ch = D.Cx + D.Cc; ch < D.Cpad; ++ch) nx[p * D.Cpad + ch] = 0;
    }
  }
}

// y = x with channels [0, C) of every NHWC bf16 pixel mapped to s*x + b (fp32 arithmetic, one rounding), the
// padded channels copied: UNetDiffusersND(center_input_sample=True)'s ``2 * x - 1.0`` on the packed model input
// (unet_diffusers_nd.py:156-157)
__global__ void affine_channels_kernel(const bf16r* __restrict__ x, int C, int Cpad, long long npix, float sc,
                                       float sh, bf16r* __restrict__ y) {
  GRID_STRIDE(i, npix * Cpad) {
    const int c = (int)(i % Cpad);
    y[i] = c < C ? (bf16r)f2bf(sc * bf2f(x[i]) + sh) : x[i];
  }
}

__global__ void counter_add_kernel(int* c, int v) {
  if (threadIdx.x == 0) c[0] += v;
}

__global__ void sum_pool2_kernel(const bf16r* __restrict__ src, int N, int H, int W, int C, bf16r* __restrict__ dst,
                                 int acc) {
  // dst[n][y][x][c] (+)= sum of the 2x2 block of src[n][2y..][2x..][c]   (dst is H x W, src 2H x 2W)
  const long long total = (long long)N * H * W * C;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int x = (int)(r % W); r /= W;
    const int y = (int)(r % H);
    const int n = (int)(r / H);
    float s = 0.f;
    for (int dy = 0; dy < 2; ++dy)
      for (int dx = 0; dx < 2; ++dx) s += bf2f(src[(((size_t)n * 2 * H + 2 * y + dy) * 2 * W + 2 * x + dx) * C + c]);
    if (acc) s += bf2f(dst[i]);
    dst[i] = (bf16r)f2bf(s);
  }
}

// Parameter-free resampling by 2 along the dims with factor 2 (1-, 2- or 3-D, NDHWC bf16, fp32 math):
//   up = 0 (AvgPoolND kernel=stride=2, src/nn/ops/pooling.py:33-53; also the nearest-x2 data gradient):
//        dst[low] (+)= scale * sum of the 2^d block of src[high] (odd high extents: the last index is dropped)
//   up = 1 (nearest-x2 F.interpolate of UpsampleND(use_conv=False), upsampling.py:24-29; also the avg-pool
//        data gradient): dst[high] (+)= scale * src[high >> 1] (0 past the low extent)
// low = (Dl, Hl, Wl), high = (Dh, Hh, Wh); a dim with factor 1 has equal extents.
__global__ void resample2_kernel(const bf16r* __restrict__ src, int N, int Dl, int Hl, int Wl, int Dh, int Hh, int Wh,
                                 int C, int fz, int fy, int fx, int up, float scale, bf16r* __restrict__ dst,
                                 int acc) {
  const long long total = (long long)N * (up ? (long long)Dh * Hh * Wh : (long long)Dl * Hl * Wl) * C;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C);
    long long r = i / C;
    if (up) {
      const int x = (int)(r % Wh); r /= Wh;
      const int y = (int)(r % Hh); r /= Hh;
      const int z = (int)(r % Dh);
      const int n = (int)(r / Dh);
      const int zl = fz == 2 ? z >> 1 : z, yl = fy == 2 ? y >> 1 : y, xl = fx == 2 ? x >> 1 : x;
      float v = 0.f;
      if (zl < Dl && yl < Hl && xl < Wl) v = scale * bf2f(src[((((size_t)n * Dl + zl) * Hl + yl) * Wl + xl) * C + c]);
      if (acc) v += bf2f(dst[i]);
      dst[i] = (bf16r)f2bf(v);
    } else {
      const int x = (int)(r % Wl); r /= Wl;
      const int y = (int)(r % Hl); r /= Hl;
      const int z = (int)(r % Dl);
      const int n = (int)(r / Dl);
      float v = 0.f;
      for (int dz = 0; dz < fz; ++dz)
        for (int dy = 0; dy < fy; ++dy)
          for (int dx = 0; dx < fx; ++dx)
            v += bf2f(src[((((size_t)n * Dh + fz * z + dz) * Hh + fy * y + dy) * Wh + fx * x + dx) * C + c]);
      v *= scale;
      if (acc) v += bf2f(dst[i]);
      dst[i] = (bf16r)f2bf(v);
    }
  }
}

__global__ void sum_pool2_3d_kernel(const bf16r* __restrict__ src, int N, int D, int H, int W, int C,
                                    bf16r* __restrict__ dst, int acc) {
  // dst[n][z][y][x][c] (+)= sum of the 2x2x2 block of src (dst D x H x W, src 2D x 2H x 2W)
  const long long total = (long long)N * D * H * W * C;
  GRID_STRIDE(i, total) {
    const int c = (int)(i % C);
    long long r = i / C;
    const int x = (int)(r % W); r /= W;
    const int y = (int)(r % H); r /= H;
    const int z = (int)(r % D);
    const int n = (int)(r / D);
    float s = 0.f;
    for (int dz = 0; dz < 2; ++dz)
      for (int dy = 0; dy < 2; ++dy)
        for (int dx = 0; dx < 2; ++dx)
          s += bf2f(src[((((size_t)n * 2 * D + 2 * z + dz) * 2 * H + 2 * y + dy) * 2 * W + 2 * x + dx) * C + c]);
    if (acc) s += bf2f(dst[i]);
    dst[i] = (bf16r)f2bf(s);
  }
}

__global__ void add_bf16_kernel(const bf16r* __restrict__ a, bf16r* __restrict__ dst, long long n) {
  GRID_STRIDE(i, n) dst[i] = (bf16r)f2bf(bf2f(dst[i]) + bf2f(a[i]));
}


// ------------------------------------------------------------------ grouped linears
// All ResBlock emb_layers (Linear(emb_dim, 2C or C), residual.py:63-68) of one UNet as ONE launch:
// the groups' output rows are concatenated ([B][sum O]); a block owns 64 rows of one group.
struct GLGroup { const float* w; const float* b; float* dw; float* db; long long O; long long off; };

// x [B][I] -> LDS (SiLU applied), 16-byte loads issued four at a time (the scalar one-load-per-iteration staging
// loop was a chain of 16 L2 round trips per block)
FMD_DEV void glinear_stage_x(const float* __restrict__ x, int n4, int in_silu, float* __restrict__ xs) {
  for (int e0 = threadIdx.x; e0 < n4; e0 += 4 * 256) {
    f32x4 v[4];
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = e0 + k * 256;
      v[k] = ((const f32x4*)x)[e < n4 ? e : 0];
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int e = e0 + k * 256;
      if (e < n4) {
        f32x4 o = v[k];
        if (in_silu) o = f32x4{siluf_(o[0]), siluf_(o[1]), siluf_(o[2]), siluf_(o[3])};
        ((f32x4*)xs)[e] = o;
      }
    }
  }
}

// A block = 64 rows of one group; 4 lanes per row, lane p reads columns p*4 + 16k.  The weight loads run in batches
// of WB (one memory latency per batch); the first batch is issued before the x staging.  Batch rows b >= B read x row
// B - 1 and are never stored.
template <int BM>
__global__ __launch_bounds__(256) void glinear_fwd_kernel(const float* __restrict__ x, int B, int I,
                                                          const GLGroup* __restrict__ G, const int2* __restrict__ blk,
                                                          int in_silu, float* __restrict__ y, int ys) {
  extern __shared__ float xs[];   // [B][I] (SiLU applied)
  constexpr int WB = 16;
  const int2 bi = blk[blockIdx.x];
  const GLGroup g = G[bi.x];
  const int lane = threadIdx.x & 63, wid = threadIdx.x >> 6;
  const int r = bi.y + wid * 16 + (lane >> 2), p = lane & 3;
  const bool act = r < g.O;
  const float* wr = g.w + (size_t)(act ? r : bi.y) * I + p * 4;   // idle lanes re-read a valid row
  f32x4 w4[WB];
  auto load = [&](int c0) {   // columns c0 + 16 j (+ p*4); c0 + 16 j < I is wave-uniform
#pragma unroll
    for (int j = 0; j < WB; ++j) w4[j] = *(const f32x4*)(wr + (c0 + 16 * j < I ? c0 + 16 * j : 0));
  };
  load(0);
  glinear_stage_x(x, B * I / 4, in_silu, xs);
  __syncthreads();
  float acc[BM];
#pragma unroll
  for (int b = 0; b < BM; ++b) acc[b] = 0.f;
  for (int c0 = 0;;) {
#pragma unroll
    for (int j = 0; j < WB; ++j) {
      const int c = c0 + 16 * j;
      if (c < I) {
#pragma unroll
        for (int b = 0; b < BM; ++b) {
          const f32x4 x4 = *(const f32x4*)(xs + min(b, B - 1) * I + c + p * 4);
          acc[b] += w4[j][0] * x4[0] + w4[j][1] * x4[1] + w4[j][2] * x4[2] + w4[j][3] * x4[3];
        }
      }
    }
    c0 += 16 * WB;
    if (c0 >= I) break;
    load(c0);
  }
#pragma unroll
  for (int b = 0; b < BM; ++b) {
    if (b < B) {
      float v = acc[b];
      v += __shfl_xor(v, 1, 64);
      v += __shfl_xor(v, 2, 64);
      if (act && p == 0) y[(size_t)b * ys + g.off + r] = v + (g.b ? g.b[r] : 0.f);
    }
  }
}

// dW[r][i] += sum_b dy[b][r] xin[b][i];  db[r] += sum_b dy[b][r];  dx partial[blk][rg][b][i] = sum_r dy[b][r] W[r][i]
// A thread owns one column quad (q) of rows rg, rg + nrg, ...; rows run in batches of RB whose weight and dW loads
// are issued together (the first batch before the staging).  dy rows are staged as [64][BM] with zeros for b >= B,
// so the unrolled batch loop needs no guard; db is one read-modify-write per row by thread rr (the per-row serial
// db update of the first form was most of its 85 us).
template <int BM>
__global__ __launch_bounds__(256) void glinear_bwd_kernel(const float* __restrict__ x, int B, int I,
                                                          const GLGroup* __restrict__ G, const int2* __restrict__ blk,
                                                          int in_silu, const float* __restrict__ dy, int dys,
                                                          float* __restrict__ part) {
  extern __shared__ float sm[];   // xin [B][I] | dy rows [64][BM]
  constexpr int RB = BM <= 8 ? 16 : 8;
  float* xs = sm;
  float* ds = sm + B * I;
  const int2 bi = blk[blockIdx.x];
  const GLGroup g = G[bi.x];
  const int nr = min(64, (int)g.O - bi.y);
  const int nq = I / 4, nrg = blockDim.x / nq;
  const int q = threadIdx.x % nq, rg = threadIdx.x / nq;
  const int i4 = q * 4;
  f32x4 w4[RB], dw4[RB];
  auto load = [&](int r0) {
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int rr = r0 + j * nrg;
      const size_t o = (size_t)(bi.y + (rr < nr ? rr : 0)) * I + i4;
      w4[j] = *(const f32x4*)(g.w + o);
      dw4[j] = *(const f32x4*)(g.dw + o);
    }
  };
  load(rg);
  glinear_stage_x(x, B * I / 4, in_silu, xs);
  for (int e = threadIdx.x; e < 64 * BM; e += blockDim.x) {
    const int rr = e / BM, b = e - rr * BM;
    ds[e] = (rr < nr && b < B) ? dy[(size_t)b * dys + g.off + bi.y + rr] : 0.f;
  }
  __syncthreads();
  if (g.db && (int)threadIdx.x < nr) {
    float sb = 0.f;
    for (int b = 0; b < B; ++b) sb += ds[threadIdx.x * BM + b];
    g.db[bi.y + threadIdx.x] += sb;
  }
  float dx[BM][4];
#pragma unroll
  for (int b = 0; b < BM; ++b) dx[b][0] = dx[b][1] = dx[b][2] = dx[b][3] = 0.f;
  for (int r0 = rg;;) {
#pragma unroll
    for (int j = 0; j < RB; ++j) {
      const int rr = r0 + j * nrg;
      if (rr >= nr) break;
      f32x4 gw = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int b = 0; b < BM; ++b) {
        const float dv = ds[rr * BM + b];
        const f32x4 x4 = *(const f32x4*)(xs + min(b, B - 1) * I + i4);
        gw += dv * x4;
#pragma unroll
        for (int e = 0; e < 4; ++e) dx[b][e] += dv * w4[j][e];
      }
      *(f32x4*)(g.dw + (size_t)(bi.y + rr) * I + i4) = dw4[j] + gw;
    }
    r0 += RB * nrg;
    if (r0 >= nr) break;
    load(r0);
  }
  float* pp = part + ((size_t)blockIdx.x * nrg + rg) * B * I;
#pragma unroll
  for (int b = 0; b < BM; ++b)
    if (b < B) *(f32x4*)(pp + (size_t)b * I + i4) = f32x4{dx[b][0], dx[b][1], dx[b][2], dx[b][3]};
}

// dx[b][i] (+)= silu'(x) * sum_p part[p][b][i].  A 1024-thread block owns 64 elements: 16 partial groups (threads
// e + 64 g) each sum partials p = g, g + 16, ... in two chains, then the groups meet in LDS in fixed order
// (deterministic).  The first form -- one thread per element walking all np (several hundred) partials -- ran on 16
// blocks for 86 us per train step.
constexpr int GLR_G = 16;
__global__ __launch_bounds__(1024) void glinear_dx_reduce(const float* __restrict__ part, int np, int B, int I,
                                                          const float* __restrict__ x, int in_silu,
                                                          float* __restrict__ dx, int acc) {
  __shared__ float red[GLR_G][64];
  const int el = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int e = blockIdx.x * 64 + el;
  const size_t BI = (size_t)B * I;
  float v0 = 0.f, v1 = 0.f;
  if (e < B * I) {
    int p = g;
    for (; p + GLR_G < np; p += 2 * GLR_G) {
      v0 += part[(size_t)p * BI + e];
      v1 += part[(size_t)(p + GLR_G) * BI + e];
    }
    if (p < np) v0 += part[(size_t)p * BI + e];
  }
  red[g][el] = v0 + v1;
  __syncthreads();
  if (g == 0 && e < B * I) {
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < GLR_G; ++k) v += red[k][el];
    if (in_silu) v *= silu_grad(x[e]);
    dx[e] = acc ? dx[e] + v : v;
  }
}

// ------------------------------------------------------------------ batched weight layouts
// One launch re-derives every bf16 kernel layout of the UNet from the fp32 masters after the
// optimizer step.  A block owns a PTK (k) x 32 (c) tile of one master weight w[K][C][T]: it reads the
// tile once (contiguous T*32-float runs per k) into LDS and writes every requested layout of it with
// contiguous 32-512 B runs.  Layouts (see fmd_prep_weights, fmd_tile_weights_halo):
//   kind 0 base: mode 0 [R=Kpad][T][Cc=Cpad]; modes 1/3 [R=Cpad][T][Cc=Kpad] (3: taps flipped);
//                mode 2 [R=Cpad][16][Cc=Kpad] (upsample + 3x3 data gradient, 4x4 effective taps)
//   kind 1 halo tiles of a base layout: [ceil(R/128)][ceil(Cc/BK)][T][BK/8][128][8], BK = FMD_HALO_BK
//   kind 2 (3x3x3 weights only) depth-packed halo tiles: the 2-D tiles of the [R][3 * Cr][3][3] view whose
//          channel block kz * Cr + c holds depth tap kz of channel c (Cr = Cc rounded up to BK), i.e.
//          [ceil(R/128)][3 * Cr / BK][9][BK/8][128][8] -- the depth-tap halo kernel's weights (modes 0, 3)
// Job (16 x int64): w, K | C << 32, ks | nout << 32, first block | kt << 32 (k tiles),
//                   then per output (<= 6): out, mode | kind << 8 | R << 16 | Cc << 40.
// TT: taps the LDS tile holds (9: ks <= 3 square kernels, T = ks * ks; 27: cubic 3x3x3 kernels, PTK = 16).
constexpr int PT = 32;          // c tile

template <int TT>
FMD_DEV float ptile_value(const float* tile, int kl, int cl, int ks, int mode, int tap) {
  constexpr int PTS = PT * TT + 1;   // LDS row stride (floats) per k: conflict-free transposed reads
  const int T = TT == 27 ? 27 : ks * ks;
  if (mode == 0 || mode == 1) return tile[kl * PTS + cl * T + tap];
  if (mode == 3) return tile[kl * PTS + cl * T + (T - 1 - tap)];
  const int ry = tap >> 2, rx = tap & 3;
  const int ylo = (ry == 0) ? 2 : (ry == 1 ? 1 : 0), yhi = (ry == 3) ? 0 : (ry == 2 ? 1 : 2);
  const int xlo = (rx == 0) ? 2 : (rx == 1 ? 1 : 0), xhi = (rx == 3) ? 0 : (rx == 2 ? 1 : 2);
  float v = 0.f;
  for (int ky = ylo; ky <= yhi; ++ky)
    for (int kx = xlo; kx <= xhi; ++kx) v += tile[kl * PTS + cl * 9 + ky * 3 + kx];
  return v;
}

template <int TT>
__global__ __launch_bounds__(256) void prep_batch_kernel(const long long* __restrict__ jobs, int njobs) {
  constexpr int PTK = TT == 27 ? 16 : 32;   // k tile
  constexpr int PTS = PT * TT + 1;
  __shared__ float tile[PTK * PTS];
  int lo = 0, hi = njobs - 1;
  while (lo < hi) {
    const int mid = (lo + hi + 1) >> 1;
    if ((jobs[mid * 16 + 3] & 0xffffffffLL) <= (long long)blockIdx.x) lo = mid; else hi = mid - 1;
  }
  const long long* J = jobs + lo * 16;
  const float* w = (const float*)J[0];
  const int K = (int)(J[1] & 0xffffffff), C = (int)(J[1] >> 32);
  const int ks = (int)(J[2] & 0xffffffff), nout = (int)(J[2] >> 32);
  const int kt = (int)(J[3] >> 32);
  const int b = (int)((long long)blockIdx.x - (J[3] & 0xffffffffLL));
  const int k0 = (b % kt) * PTK, c0 = (b / kt) * PT;
  const int T = TT == 27 ? 27 : ks * ks;
  // ---- master tile w[k0:k0+PTK][c0:c0+32][:] (zero outside K x C)
  if (((C * T) & 3) == 0 && c0 + PT <= C && ((size_t)w & 15) == 0) {
    // full-width tile: 16-byte loads along the contiguous (c, tap) run of each k
    const int nv = PT * T / 4;
    for (int e = threadIdx.x; e < PTK * nv; e += blockDim.x) {
      const int kl = e / nv, v = e - kl * nv, k = k0 + kl;
      const float4 x = k < K ? *(const float4*)(w + ((size_t)k * C + c0) * T + v * 4) : float4{0.f, 0.f, 0.f, 0.f};
      float* t = tile + kl * PTS + v * 4;
      t[0] = x.x; t[1] = x.y; t[2] = x.z; t[3] = x.w;
    }
  } else {
    for (int e = threadIdx.x; e < PTK * PT * T; e += blockDim.x) {
      const int kl = e / (PT * T), r = e - kl * (PT * T);   // r = cl * T + tap: contiguous in memory
      const int k = k0 + kl, c = c0 + r / T;
      tile[kl * PTS + r] = (k < K && c < C) ? w[((size_t)k * C + c0) * T + r] : 0.f;
    }
  }
  __syncthreads();
  for (int o = 0; o < nout; ++o) {
    bf16r* out = (bf16r*)J[4 + 2 * o];
    const long long desc = J[5 + 2 * o];
    const int mode = (int)(desc & 0xff), kind = (int)((desc >> 8) & 0xff);
    const int R = (int)((desc >> 16) & 0xffffff), Cc = (int)((desc >> 40) & 0xffffff);
    const int To = mode == 2 ? 16 : T;
    // tile coordinates in the layout's (row, col) space: NRB rows x NCB cols of this block
    const int r0 = mode == 0 ? k0 : c0, q0 = mode == 0 ? c0 : k0;
    const int NRB = mode == 0 ? PTK : PT, NCB = mode == 0 ? PT : PTK;
    if (kind == 0) {
      // [R][To][Cc]: for each (row, tap) a run of NCB cols, written as 16-byte groups of 8
      const bool vec = (Cc & 7) == 0 && ((size_t)out & 15) == 0;
      for (int e = threadIdx.x; e < NRB * To * (NCB / 8); e += blockDim.x) {
        const int q8 = e % (NCB / 8), r = e / (NCB / 8), tap = r % To, rl = r / To;
        const int row = r0 + rl, col8 = q0 + q8 * 8;
        if (row >= R || col8 >= Cc) continue;
        bf16r* dst = out + ((size_t)row * To + tap) * Cc + col8;
        if (vec) {
          unsigned int pk[4];
#pragma unroll
          for (int h = 0; h < 4; ++h) {
            float v2[2];
#pragma unroll
            for (int u = 0; u < 2; ++u) {
              const int ql = q8 * 8 + 2 * h + u;
              const int kl = mode == 0 ? rl : ql, cl = mode == 0 ? ql : rl;
              v2[u] = ptile_value<TT>(tile, kl, cl, ks, mode, tap);
            }
            pk[h] = pack2(v2[0], v2[1]);
          }
          *(u32x4*)dst = u32x4{pk[0], pk[1], pk[2], pk[3]};
        } else {
          for (int u = 0; u < 8 && col8 + u < Cc; ++u) {
            const int ql = q8 * 8 + u;
            const int kl = mode == 0 ? rl : ql, cl = mode == 0 ? ql : rl;
            dst[u] = (bf16r)f2bf(ptile_value<TT>(tile, kl, cl, ks, mode, tap));
          }
        }
      }
    } else {
      // kind 1: [R/128][Cc/BK][To][BK/8][128][8]; kind 2: [R/128][3 * Cc/BK][9][BK/8][128][8] (chunk kz * nchunk + c / BK,
      // tap9 = tap % 9): 16-byte chunks of 8 cols, runs of NRB rows
      constexpr int HBK = FMD_HALO_BK;
      const int nchunk = (Cc + HBK - 1) / HBK;
      for (int e = threadIdx.x; e < To * (NCB / 8) * NRB; e += blockDim.x) {
        const int rl = e % NRB, r = e / NRB, kq = r % (NCB / 8), tap = r / (NCB / 8);
        const int row = r0 + rl, col8 = q0 + kq * 8;
        if (row >= ((R + 127) / 128) * 128 || col8 >= nchunk * HBK) continue;
        const int tr = row >> 7, co = row & 127, chunk = col8 / HBK, kc = (col8 % HBK) >> 3;
        unsigned int pk[4];
#pragma unroll
        for (int h = 0; h < 4; ++h) {
          float v2[2];
#pragma unroll
          for (int u = 0; u < 2; ++u) {
            const int ql = kq * 8 + 2 * h + u, col = q0 + ql;
            const int kl = mode == 0 ? rl : ql, cl = mode == 0 ? ql : rl;
            v2[u] = (row < R && col < Cc) ? ptile_value<TT>(tile, kl, cl, ks, mode, tap) : 0.f;
          }
          pk[h] = pack2(v2[0], v2[1]);
        }
        size_t idx;
        if (kind == 1) {
          idx = ((((size_t)tr * nchunk + chunk) * To + tap) * (HBK / 8) + kc) * 128 + co;
        } else {
          const int kz = tap / 9, t9 = tap - kz * 9;
          idx = ((((size_t)tr * 3 * nchunk + kz * nchunk + chunk) * 9 + t9) * (HBK / 8) + kc) * 128 + co;
        }
        *(u32x4*)(out + idx * 8) = u32x4{pk[0], pk[1], pk[2], pk[3]};
      }
    }
  }
}

}  // namespace

#define LAUNCH(kernel, grid, ...)                                                   \
  do {                                                                              \
    hipLaunchKernelGGL(kernel, dim3(grid), dim3(256), 0, (hipStream_t)s, __VA_ARGS__); \
    return (int)hipGetLastError();                                                  \
  } while (0)

extern "C" {

int fmd_prep_weights(const float* w, int32_t K, int32_t C, int32_t ks, int32_t mode, int32_t Kpad, int32_t Cpad,
                      void* out, fmd_stream_t s) {
  const long long total = (long long)Kpad * Cpad * (mode == 2 ? 16 : ks * ks);
  LAUNCH(prep_weights_kernel, grid_for(total), w, K, C, ks, ks * ks, mode, Kpad, Cpad, (bf16r*)out);
}

int fmd_prep_weights_t(const float* w, int32_t K, int32_t C, int32_t T, int32_t mode, int32_t Kpad, int32_t Cpad,
                       void* out, fmd_stream_t s) {
  if (mode != 0 && mode != 1 && mode != 3) return -1;
  if (T < 1 || K > Kpad || C > Cpad) return -2;
  const long long total = (long long)Kpad * Cpad * T;
  LAUNCH(prep_weights_kernel, grid_for(total), w, K, C, 0, T, mode, Kpad, Cpad, (bf16r*)out);
}


int fmd_prep_weights_batch(const void* jobs, int32_t njobs, int32_t nblocks, fmd_stream_t s) {
  if (njobs < 1 || nblocks < 1) return njobs == 0 ? 0 : -1;
  hipLaunchKernelGGL(prep_batch_kernel<9>, dim3(nblocks), dim3(256), 0, (hipStream_t)s, (const long long*)jobs,
                     njobs);
  return (int)hipGetLastError();
}

int fmd_prep_weights_batch_cubic(const void* jobs, int32_t njobs, int32_t nblocks, fmd_stream_t s) {
  if (njobs < 1 || nblocks < 1) return njobs == 0 ? 0 : -1;
  hipLaunchKernelGGL(prep_batch_kernel<27>, dim3(nblocks), dim3(256), 0, (hipStream_t)s, (const long long*)jobs,
                     njobs);
  return (int)hipGetLastError();
}

int fmd_nchw_to_nhwc(const float* x, int32_t N, int32_t C, int32_t HW, int32_t Cpad, void* y, fmd_stream_t s) {
  LAUNCH(nchw_to_nhwc_kernel, grid_for((long long)N * HW * Cpad), x, N, C, HW, Cpad, (bf16r*)y);
}

int fmd_nhwc_to_nchw(const void* y, int32_t src_f32, int32_t N, int32_t C, int32_t HW, int32_t Cs, float* x,
                      fmd_stream_t s) {
  LAUNCH(nhwc_to_nchw_kernel, grid_for((long long)N * HW * C), y, src_f32, N, C, HW, Cs, x);
}


int fmd_timestep_embedding(const float* t, int32_t N, int32_t dim, int32_t flip, int32_t shift, float max_period,
                           float t_scale, int32_t t_trunc, float* out, fmd_stream_t s) {
  const float nlp = -(float)log((double)max_period);
  LAUNCH(temb_kernel, grid_for((long long)N * dim), t, N, dim, flip, shift, nlp, t_scale, t_trunc, out);
}

int fmd_linear(const float* x, int32_t B, int32_t I, const float* w, const float* b, int32_t O, int32_t in_silu,
               float* y, int32_t y_stride, fmd_stream_t s) {
  if (B < 1 || B > 32) return -1;
  if (B <= 8) {
    LAUNCH(linear_kernel<8>, (O + 3) / 4, x, B, I, w, b, O, in_silu, y, y_stride);
  } else {
    LAUNCH(linear_kernel<32>, (O + 3) / 4, x, B, I, w, b, O, in_silu, y, y_stride);
  }
}

int fmd_grouped_linear(const float* x, int32_t B, int32_t I, const void* groups, const void* blocks, int32_t nblk,
                       int32_t in_silu, float* y, int32_t y_stride, fmd_stream_t s) {
  if (B < 1 || B > 32 || I % 16 || (size_t)B * I * 4 > 64 * 1024) return -1;
  auto* kern = B <= 8 ? glinear_fwd_kernel<8> : glinear_fwd_kernel<32>;
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), (size_t)B * I * 4, (hipStream_t)s, x, B, I, (const GLGroup*)groups,
                     (const int2*)blocks, in_silu, y, y_stride);
  return (int)hipGetLastError();
}

int64_t fmd_grouped_linear_bwd_workspace(int32_t B, int32_t I, int32_t nblk) {
  return (int64_t)nblk * (1024 / I) * B * I;
}

int fmd_grouped_linear_bwd(const float* x, int32_t B, int32_t I, const void* groups, const void* blocks,
                           int32_t nblk, int32_t in_silu, const float* dy, int32_t dy_stride, float* dx,
                           int32_t dx_acc, float* ws, fmd_stream_t s) {
  if (B < 1 || B > 32 || (I != 128 && I != 256 && I != 512 && I != 1024)) return -1;
  const int bm = B <= 8 ? 8 : 32;
  const size_t lds = (size_t)(B * I + 64 * bm) * 4;
  if (lds > 64 * 1024) return -1;
  auto* kern = bm == 8 ? glinear_bwd_kernel<8> : glinear_bwd_kernel<32>;
  hipLaunchKernelGGL(kern, dim3(nblk), dim3(256), lds, (hipStream_t)s, x, B, I, (const GLGroup*)groups,
                     (const int2*)blocks, in_silu, dy, dy_stride, ws);
  int rc = (int)hipGetLastError();
  if (rc || !dx) return rc;
  hipLaunchKernelGGL(glinear_dx_reduce, dim3((B * I + 63) / 64), dim3(1024), 0, (hipStream_t)s, ws,
                     nblk * (1024 / I), B, I, x, in_silu, dx, dx_acc);
  return (int)hipGetLastError();
}

int fmd_linear_bwd(const float* x, int32_t B, int32_t I, const float* w, int32_t O, int32_t in_silu,
                   const float* dy, int32_t dy_stride, float* dx, int32_t dx_acc, float* dw, float* db,
                   fmd_stream_t s) {
  if (dw) {
    hipLaunchKernelGGL(linear_dw_kernel, dim3(grid_for((long long)O * I)), dim3(256), 0, (hipStream_t)s, x, B, I, O,
                       in_silu, dy, dy_stride, dw, db);
    int rc = (int)hipGetLastError();
    if (rc) return rc;
  }
  if (dx) {
    if (B > 32 || (size_t)O * 4 > 48 * 1024) return -1;
    hipLaunchKernelGGL(linear_dx_kernel, dim3((I + 63) / 64, B), dim3(256), (size_t)O * 4, (hipStream_t)s, x, B, I,
                       w, O, in_silu, dy, dy_stride, dx, dx_acc);
    return (int)hipGetLastError();
  }
  return 0;
}

int fmd_silu_bwd_f32(const float* x, const float* dy, float* dx, int64_t n, fmd_stream_t s) {
  LAUNCH(silu_bwd_kernel, grid_for(n), x, dy, dx, (long long)n);
}

int fmd_noise_prepare(const float* x0, const float* noise, const float* ca, const float* cb, const float* cond,
                      int32_t N, int32_t HW, int32_t Cx, int32_t Cc, int32_t Cpad, void* inp, fmd_stream_t s) {
  LAUNCH(noise_prepare_kernel, grid_for((long long)N * HW * Cpad), x0, noise, ca, cb, cond, N, HW, Cx, Cc, Cpad,
         (bf16r*)inp);
}

int fmd_add_noise(const float* x0, const float* noise, const float* sqrt_acp, const float* sqrt_1m_acp,
                  const int64_t* timesteps, int32_t N, int64_t per_sample, float* out, fmd_stream_t s) {
  if (N <= 0 || per_sample <= 0) return N == 0 ? 0 : -1;
  LAUNCH(add_noise_kernel, grid_for((long long)N * per_sample), x0, noise, sqrt_acp, sqrt_1m_acp,
         (const long long*)timesteps, (long long)per_sample, N, out);
}

int fmd_mse(const float* pred, int32_t Kpad, const float* ta, const float* tb, float tb_sign, int32_t N, int32_t Cx,
            int32_t HW, float grad_scale, float* partial, int32_t max_blocks, float* loss, void* dpred,
            fmd_stream_t s) {
  const long long total = (long long)N * HW * Kpad;
  int blocks = grid_for(total, 256, max_blocks);
  const float inv = 1.f / (float)((long long)N * Cx * HW);
  hipLaunchKernelGGL(mse_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)s, pred, Kpad, ta, tb, tb_sign, N, Cx, HW,
                     inv, grad_scale, partial, (bf16r*)dpred);
  int rc = (int)hipGetLastError();
  if (rc) return rc;
  hipLaunchKernelGGL(sum_partials_kernel, dim3(1), dim3(256), 0, (hipStream_t)s, partial, blocks, inv, loss);
  return (int)hipGetLastError();
}

int fmd_adamw(float* p, const float* g, float* m, float* v, int64_t n, float lr, float beta1, float beta2, float eps,
              float wd, float bc1, float bc2, fmd_stream_t s) {
  LAUNCH(adamw_kernel, grid_for(n, 256, 8192), p, g, m, v, (long long)n, lr, beta1, beta2, eps, wd, bc1, sqrtf(bc2));
}

int fmd_adamw_sched(float* p, const float* g, float* m, float* v, int64_t n, const int32_t* step_ctr, float base_lr,
                    int32_t warmup, int32_t total, float beta1, float beta2, float eps, float wd, float grad_scale,
                    fmd_stream_t s) {
  const int vec = ((reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                    reinterpret_cast<uintptr_t>(v)) & 15) == 0;
  LAUNCH(adamw_sched_kernel, grid_for(vec ? n / 4 : n, 256, 8192), p, g, m, v, (long long)n, step_ctr, base_lr, warmup,
         total, beta1, beta2, eps, wd, grad_scale, vec);
}

int fmd_flow_euler(float* x, const float* v, int32_t Kpad, const float* sigmas, const int32_t* index, int32_t N,
                   int32_t Cx, int32_t HW, const float* cond, int32_t Cc, int32_t Cpad, void* next, fmd_stream_t s) {
  LAUNCH(flow_euler_kernel, grid_for((long long)N * HW), x, v, Kpad, sigmas, index, N, Cx, HW, cond, Cc, Cpad,
         (bf16r*)next);
}

int fmd_ddpm_step(float* x, const float* eps, int32_t Kpad, const float* coef, const int32_t* index,
                  const float* noise, int32_t noise_base, int32_t N, int32_t Cx, int32_t HW, const float* cond,
                  int32_t Cc, int32_t Cpad, void* next, fmd_stream_t s) {
  LAUNCH(ddpm_step_kernel, grid_for((long long)N * HW), x, eps, Kpad, coef, index, noise, noise_base, N, Cx, HW, cond,
         Cc, Cpad,
         (bf16r*)next);
}

int fmd_fill_from_table(const float* table, const int32_t* index, float* out, int32_t N, fmd_stream_t s) {
  if (N > 256) return -1;
  LAUNCH(fill_from_table_kernel, 1, table, index, out, N);
}

int fmd_counter_add(int32_t* c, int32_t v, fmd_stream_t s) { LAUNCH(counter_add_kernel, 1, c, v); }

int fmd_affine_channels(const void* x, int32_t C, int32_t Cpad, int64_t npix, float scale, float shift, void* y,
                        fmd_stream_t s) {
  if (!x || !y || C < 0 || C > Cpad || npix < 0) return -1;
  LAUNCH(affine_channels_kernel, grid_for(npix * Cpad), (const bf16r*)x, C, Cpad, (long long)npix, scale, shift,
         (bf16r*)y);
}

int fmd_lincomb(const fmd_lincomb_desc* d, fmd_stream_t s) {
  if (!d || !d->out || d->nin < 1 || d->nin > FMD_LINCOMB_MAX || d->n < 0) return -1;
  for (int k = 0; k < d->nin; ++k)
    if (!d->in[k]) return -2;
  if ((d->n & 3) == 0) {
    if (((size_t)d->out & 15) != 0) return -3;
    for (int k = 0; k < d->nin; ++k)
      if (((size_t)d->in[k] & 15) != 0) return -3;
  }
  if (d->n == 0) return 0;
  LAUNCH(lincomb_kernel, grid_for((d->n & 3) == 0 ? d->n / 4 : d->n), *d);
}

int fmd_sched_step(const fmd_sched_step_desc* d, fmd_stream_t s) {
  if (!d || !d->x || !d->eps || !d->coef || !d->index || d->N < 1 || d->Cx < 1 || d->HW < 1 || d->Kpad < d->Cx)
    return -1;
  for (int k = 0; k < 4; ++k)
    if (!d->ring[k]) return -2;
  if (d->next && (d->Cpad < d->Cx + d->Cc || (d->Cc > 0 && !d->cond))) return -3;
  LAUNCH(sched_step_kernel, grid_for((long long)d->N * d->HW), *d);
}

int fmd_gather_row(const float* table, const int32_t* index, int64_t n, float* out, fmd_stream_t s) {
  if (n < 1 || !table || !index || !out) return -1;
  LAUNCH(gather_row_kernel, grid_for(n), table, index, (long long)n, out);
}

int fmd_sum_pool2(const void* src, int32_t N, int32_t H, int32_t W, int32_t C, void* dst, int32_t acc,
                  fmd_stream_t s) {
  LAUNCH(sum_pool2_kernel, grid_for((long long)N * H * W * C), (const bf16r*)src, N, H, W, C, (bf16r*)dst, acc);
}

int fmd_sum_pool2_3d(const void* src, int32_t N, int32_t D, int32_t H, int32_t W, int32_t C, void* dst,
                     int32_t acc, fmd_stream_t s) {
  LAUNCH(sum_pool2_3d_kernel, grid_for((long long)N * D * H * W * C), (const bf16r*)src, N, D, H, W, C,
         (bf16r*)dst, acc);
}

int fmd_resample2(const void* src, int32_t N, int32_t Dl, int32_t Hl, int32_t Wl, int32_t Dh, int32_t Hh, int32_t Wh,
                  int32_t C, int32_t fz, int32_t fy, int32_t fx, int32_t up, float scale, void* dst, int32_t acc,
                  fmd_stream_t s) {
  if (N < 1 || C < 1 || Dl < 1 || Hl < 1 || Wl < 1 || fz < 1 || fz > 2 || fy < 1 || fy > 2 || fx < 1 || fx > 2)
    return -1;
  if (Dh < fz * Dl || Hh < fy * Hl || Wh < fx * Wl || Dh > fz * Dl + 1 || Hh > fy * Hl + 1 || Wh > fx * Wl + 1)
    return -1;
  const long long work = (long long)N * (up ? (long long)Dh * Hh * Wh : (long long)Dl * Hl * Wl) * C;
  LAUNCH(resample2_kernel, grid_for(work), (const bf16r*)src, N, Dl, Hl, Wl, Dh, Hh, Wh, C, fz, fy, fx, up, scale,
         (bf16r*)dst, acc);
}

int fmd_add_bf16(const void* a, void* dst, int64_t n, fmd_stream_t s) {
  LAUNCH(add_bf16_kernel, grid_for(n), (const bf16r*)a, (bf16r*)dst, (long long)n);
}

}  // extern "C"
