// Weight-gradient GEMM for the implicit-GEMM convolutions (gfx950).
//
// dW[cout][tap][cin] = sum_p dY[p][cout] * G[p][tap][cin], reduction over the
// pixels p = N*Ho*Wo.  Both operands are pixel-major in HBM (NHWC), so the
// reduction dimension is the strided one: tiles are staged [pixel][channel] in
// LDS and read as MFMA fragments with gfx950's transposing ds_read_b64_tr_b16
// (two reads give the 8 consecutive pixels a 16x16x32 fragment lane holds).
// G is the same gather + GroupNorm-affine/SiLU prologue as the forward, so the
// activations of the forward are recomputed on the fly, never stored.
// The pixel range is split across workgroups (split-K); partial slabs are
// reduced deterministically by a second kernel that writes the reference's
// [K][C][kh][kw] fp32 layout.  The bias gradient (sum of dY) rides along.
//
// Replaces: autograd of nn.Conv2d weight/bias (src/nn/ops/convolution.py:53).
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

constexpr int BCO = 128, BCI = 128, BKP = 32;

struct WArgs {
  fmd_wgrad_desc d;
  int M, T, C, ntc, nci, per_split, nsteps, ldy;
  int merged;   // C < BCI: the column tiles run over the flattened (tap, cin) pairs (narrow convs: the stem, the
                // 3-D input conv with 27 taps x 8 channels = 2 tiles instead of 27 tiles of 8 valid columns)
};

// 8-byte unit swizzle for the [32][128] bf16 tile (256-B rows): conflict-free
// transposed reads for the 4-row blocks rows {8g+q} read by one instruction.
FMD_DEV int swz(int row) { return 4 * ((row & 3) | (((row >> 3) & 1) << 2)); }
FMD_DEV int lds_off(int row, int unit) { return row * 128 + 4 * (unit ^ swz(row)); }  // in bf16 elements

__global__ __launch_bounds__(256, 2) void wgrad_kernel(const WArgs A) {
  __shared__ __attribute__((aligned(16))) bf16r lds[2][2][BKP * 128];
  __shared__ float bsum[4][BCO];
  const fmd_wgrad_desc& d = A.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wm = wid >> 1, wn = wid & 1;

  // grid: x = (co tile, tap, ci tile), y = split
  int bx = blockIdx.x;
  const int tco = bx % A.ntc; bx /= A.ntc;
  const int tci = bx % A.nci; bx /= A.nci;
  const int tap = bx;
  const int co0 = tco * BCO, ci0 = tci * BCI;
  // this thread's gather column chunk -> (tap, channel); merged mode spreads the taps over the chunks
  const int cpt = A.C >> 3;                        // 8-channel chunks per tap
  const int qc = tci * (BCI / 8) + (tid & 15);     // merged: flattened (tap, chunk) index of this column chunk
  const int my_tap = A.merged ? qc / cpt : tap;
  const int my_c = A.merged ? (qc - my_tap * cpt) * 8 : ci0 + (tid & 15) * 8;
  const bool col_ok = A.merged ? my_tap < A.T : my_c < A.C;
  const int kk2 = d.ks * d.ks;
  const int kz = my_tap / kk2, t2 = my_tap - (my_tap / kk2) * kk2;   // kz = 0 in 2-D
  const int ky = t2 / d.ks, kx = t2 - (t2 / d.ks) * d.ks;
  const bool d3 = d.Do > 0;
  const int Dsz = d.Ds > 0 ? d.Ds : 1, Dz = d.Do > 0 ? d.Do : 1;
  const int split = blockIdx.y;
  const int s0 = split * A.per_split;
  const int s1 = min(A.nsteps, s0 + A.per_split);
  const bool do_bias = d.db && tap == 0 && tci == 0;

  const int HWo = Dz * d.Ho * d.Wo, HWs = d.Ho * d.Wo;
  const int chunk = tid & 15;     // 8-channel chunk
  const int rb = tid >> 4;        // row (pixel) 0..15, +16
  const bf16r* __restrict__ dy = (const bf16r*)d.dy;
  const bf16r* __restrict__ x0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ x1 = (const bf16r*)d.src1;
  const bool pro = d.pro_a != nullptr;

  u32x4 ry[2], rg[2];
  bool vg[2];
  int gn[2];
  float bacc[8];
#pragma unroll
  for (int e = 0; e < 8; ++e) bacc[e] = 0.f;

  auto load = [&](int step) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int p = step * BKP + rb + 16 * j;
      const int co = co0 + chunk * 8;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (p < A.M && co < d.K) v = *(const u32x4*)(dy + (size_t)p * A.ldy + co);
      ry[j] = v;
      // gather
      const int c = my_c;
      bool ok = p < A.M && col_ok;
      int n = 0;
      const bf16r* ptr = nullptr;
      if (ok) {
        n = p / HWo;
        int rem = p - n * HWo;
        const int oz = rem / HWs;
        rem -= oz * HWs;
        const int oy = rem / d.Wo, ox = rem - (rem / d.Wo) * d.Wo;
        const int iz = d3 ? oz * d.stride + kz - d.pad : 0;
        const int iy = oy * d.stride + ky - d.pad, ix = ox * d.stride + kx - d.pad;
        int sz, sy, sx;
        if (d.upsample) {
          ok = iy >= 0 && iy < 2 * d.Hs && ix >= 0 && ix < 2 * d.Ws && iz >= 0 && iz < 2 * Dsz;
          sz = iz >> 1; sy = iy >> 1; sx = ix >> 1;
        } else {
          ok = iy >= 0 && iy < d.Hs && ix >= 0 && ix < d.Ws && iz >= 0 && iz < Dsz;
          sz = iz; sy = iy; sx = ix;
        }
        if (ok) {
          const size_t pix = (((size_t)n * Dsz + sz) * d.Hs + sy) * d.Ws + sx;
          ptr = (c < d.C0) ? x0 + pix * d.C0 + c : x1 + pix * d.C1 + (c - d.C0);
        }
      }
      vg[j] = ok;
      gn[j] = n;
      rg[j] = ok ? *(const u32x4*)ptr : u32x4{0u, 0u, 0u, 0u};
    }
  };

  auto transform = [&](int step) {
    (void)step;
    if (do_bias) {
#pragma unroll
      for (int j = 0; j < 2; ++j)
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          bacc[2 * e] += bf_lo(ry[j][e]);
          bacc[2 * e + 1] += bf_hi(ry[j][e]);
        }
    }
    if (!pro) return;
    const int c = my_c;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      if (!vg[j]) continue;
      const float* pa = d.pro_a + (size_t)gn[j] * A.C + c;
      const float* pb = d.pro_b + (size_t)gn[j] * A.C + c;
      const f32x4 a0 = *(const f32x4*)pa, a1 = *(const f32x4*)(pa + 4);
      const f32x4 b0 = *(const f32x4*)pb, b1 = *(const f32x4*)(pb + 4);
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = bf_lo(rg[j][e]) * av[2 * e] + bv[2 * e];
        float hi = bf_hi(rg[j][e]) * av[2 * e + 1] + bv[2 * e + 1];
        if (d.pro_silu) { lo = siluf_(lo); hi = siluf_(hi); }
        o[e] = pack2(lo, hi);
      }
      rg[j] = o;
    }
  };

  auto store = [&](int buf) {
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int r = rb + 16 * j;
      *(u32x4*)(&lds[buf][0][lds_off(r, 2 * chunk)]) = ry[j];
      *(u32x4*)(&lds[buf][1][lds_off(r, 2 * chunk)]) = rg[j];
    }
  };

  f32x4 acc[4][4];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int g = lane >> 4, q = (lane >> 2) & 3, pp = lane & 3;
  auto frag = [&](const bf16r* t, int col0) -> bf16x8 {
    // rows 8g+q (first) and 8g+4+q (second); cols col0 + 4pp
    const s16x4 lo = ds_read_tr16(t + lds_off(8 * g + q, col0 / 4 + pp));
    const s16x4 hi = ds_read_tr16(t + lds_off(8 * g + 4 + q, col0 / 4 + pp));
    typedef __attribute__((ext_vector_type(8))) short s16x8;
    s16x8 v = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  auto compute = [&](int buf) {
    bf16x8 af[4], bfr[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = frag(lds[buf][0], wm * 64 + 16 * i);
#pragma unroll
    for (int j = 0; j < 4; ++j) bfr[j] = frag(lds[buf][1], wn * 64 + 16 * j);
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
  };

  if (s0 < s1) {
    load(s0);
    transform(s0);
    store(0);
    __syncthreads();
    for (int st = s0; st < s1; ++st) {
      const int buf = (st - s0) & 1;
      const bool nxt = st + 1 < s1;
      if (nxt) load(st + 1);
      compute(buf);
      if (nxt) {
        transform(st + 1);
        store(buf ^ 1);
      }
      __syncthreads();
    }
  }

  // partial slab: ws[split][co][tap][ci]
  float* ws = d.ws + (size_t)split * d.K * A.T * A.C;
  const int l16 = lane & 15, lq = lane >> 4;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int col = wn * 64 + 16 * j + l16;
      const int fq = tci * BCI + col;   // merged: flattened (tap, cin) column
      const int ci = A.merged ? fq % A.C : ci0 + col;
      const int ct = A.merged ? fq / A.C : tap;
      if (A.merged ? ct >= A.T : ci >= A.C) continue;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wm * 64 + 16 * i + 4 * lq + r;
        if (co < d.K) ws[((size_t)co * A.T + ct) * A.C + ci] = acc[i][j][r];
      }
    }
  }
  if (do_bias) {
    // rows share a chunk at lane stride 16 within a wave, then across waves via LDS
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      float v = bacc[e];
      v += __shfl_xor(v, 16, 64);
      v += __shfl_xor(v, 32, 64);
      bacc[e] = v;
    }
    if (lane < 16) {
#pragma unroll
      for (int e = 0; e < 8; ++e) bsum[wid][chunk * 8 + e] = bacc[e];
    }
    __syncthreads();
    if (tid < BCO && co0 + tid < d.K) {
      float* wb = d.ws + (size_t)gridDim.y * d.K * A.T * A.C + (size_t)split * d.K;
      wb[co0 + tid] = bsum[0][tid] + bsum[1][tid] + bsum[2][tid] + bsum[3][tid];
    }
  }
}

// Sum the split-K slabs ws[s*sstride][k][tap][c] (s < nsl) and write the reference layout dW[k][c][tap]
// (+ db from the same, possibly pre-reduced, bias slabs).  A block owns (k, 64 channels): it reads
// [tap][64 c] runs and writes the contiguous dW[k][c0:c0+64][:] run through LDS.
constexpr int RC = 64;

__global__ __launch_bounds__(256) void wgrad_reduce(const WArgs A, int splits, int nsl, int sstride) {
  const fmd_wgrad_desc& d = A.d;
  __shared__ float res[RC * 27 + 1];   // [c][tap], T <= 27 (3x3x3)
  const size_t per = (size_t)d.K * A.T * A.C;
  const int k = blockIdx.x, c0 = blockIdx.y * RC;
  const int nc = min(RC, A.C - c0);
  const int n = A.T * RC;
  for (int e = threadIdx.x; e < n; e += blockDim.x) {
    const int tap = e / RC, cl = e - tap * RC;
    if (cl >= nc) continue;
    const size_t src = ((size_t)k * A.T + tap) * A.C + c0 + cl;
    float v0 = 0.f, v1 = 0.f, v2 = 0.f, v3 = 0.f;
    int s = 0;
    for (; s + 4 <= nsl; s += 4) {
      v0 += d.ws[(size_t)s * sstride * per + src];
      v1 += d.ws[(size_t)(s + 1) * sstride * per + src];
      v2 += d.ws[(size_t)(s + 2) * sstride * per + src];
      v3 += d.ws[(size_t)(s + 3) * sstride * per + src];
    }
    for (; s < nsl; ++s) v0 += d.ws[(size_t)s * sstride * per + src];
    res[cl * A.T + tap] = (v0 + v1) + (v2 + v3);
  }
  __syncthreads();
  float* out = d.dw + ((size_t)k * A.C + c0) * A.T;
  for (int e = threadIdx.x; e < nc * A.T; e += blockDim.x) out[e] = d.accumulate ? out[e] + res[e] : res[e];
  if (d.db && blockIdx.y == 0 && threadIdx.x == 0) {
    const float* wb = d.ws + (size_t)splits * per;
    float v = 0.f;
    for (int s = 0; s < nsl; ++s) v += wb[(size_t)s * sstride * d.K + k];
    d.db[k] = d.accumulate ? d.db[k] + v : v;
  }
}

// Combine with all T taps of (k, 64 channels) per block and the slabs spread over SL slab lanes, so every form
// of the problem keeps the block busy: items (tap, 4-channel quad) x SL lanes <= 512 threads, each lane summing
// slabs sl, sl + SL, ... (of the nsl slabs at stride sstride) as 16-byte loads in four chains; the lanes are then
// combined in fixed order through LDS and written transposed to the reference dW[k][c][tap] layout.
// Deterministic.  T <= 27, C % 4 == 0, blockDim 512.
__global__ __launch_bounds__(512) void wgrad_reduce2(const WArgs A, int splits, int nsl, int sstride, int SL) {
  const fmd_wgrad_desc& d = A.d;
  __shared__ __attribute__((aligned(16))) float part[512 * 4];   // [sl][tap][64 c]
  const size_t per = (size_t)d.K * A.T * A.C;
  const int k = blockIdx.x, c0 = blockIdx.y * RC;
  const int items = 16 * A.T;
  const int t = threadIdx.x;
  if (t < items * SL) {
    const int sl = t / items, it = t - sl * items;
    const int tap = it >> 4, cq = it & 15;
    const int c = c0 + cq * 4;
    f32x4 a0 = {0.f, 0.f, 0.f, 0.f}, a1 = a0, a2 = a0, a3 = a0;
    if (c < A.C) {
      const float* src = d.ws + ((size_t)k * A.T + tap) * A.C + c;
      const size_t st = (size_t)SL * sstride * per;
      const float* p = src + (size_t)sl * sstride * per;
      int s = sl;
      for (; s + 3 * SL < nsl; s += 4 * SL, p += 4 * st) {
        a0 += *(const f32x4*)p;
        a1 += *(const f32x4*)(p + st);
        a2 += *(const f32x4*)(p + 2 * st);
        a3 += *(const f32x4*)(p + 3 * st);
      }
      for (; s < nsl; s += SL, p += st) a0 += *(const f32x4*)p;
    }
    *(f32x4*)&part[((size_t)sl * A.T + tap) * 64 + cq * 4] = (a0 + a1) + (a2 + a3);
  }
  __syncthreads();
  const int nc = min(RC, A.C - c0);
  float* out = d.dw + ((size_t)k * A.C + c0) * A.T;
  for (int e = t; e < nc * A.T; e += blockDim.x) {
    const int cl = e / A.T, tap = e - cl * A.T;
    float v = part[tap * 64 + cl];
    for (int sl = 1; sl < SL; ++sl) v += part[((size_t)sl * A.T + tap) * 64 + cl];
    out[e] = d.accumulate ? out[e] + v : v;
  }
  if (d.db && blockIdx.y == 0 && t < 64) {
    const float* wb = d.ws + (size_t)splits * per;
    float v = 0.f;
    for (int s = t; s < nsl; s += 64) v += wb[(size_t)s * sstride * d.K + k];
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m, 64);
    if (t == 0) d.db[k] = d.accumulate ? d.db[k] + v : v;
  }
}

WArgs make_args(const fmd_wgrad_desc* d) {
  WArgs A;
  A.d = *d;
  A.M = d->N * (d->Do > 0 ? d->Do : 1) * d->Ho * d->Wo;
  A.T = d->ks * d->ks * (d->Do > 0 ? d->ks : 1);
  A.C = d->C0 + d->C1;
  A.ntc = (d->K + BCO - 1) / BCO;
  A.nci = (A.C + BCI - 1) / BCI;
  A.nsteps = (A.M + BKP - 1) / BKP;
  A.ldy = d->ldy > 0 ? d->ldy : d->K;
  const int splits = d->splits > 1 ? d->splits : 1;
  A.per_split = (A.nsteps + splits - 1) / splits;
  A.merged = A.T > 1 && A.C < BCI;
  if (A.merged) A.nci = (A.T * A.C + BCI - 1) / BCI;   // column tiles of flattened (tap, cin) pairs
  return A;
}

}  // namespace

extern "C" int64_t fmd_wgrad_workspace(const fmd_wgrad_desc* d) {
  const int splits = d->splits > 1 ? d->splits : 1;
  const int64_t C = d->C0 + d->C1;
  const int64_t T = (int64_t)d->ks * d->ks * (d->Do > 0 ? d->ks : 1);
  return (int64_t)splits * d->K * T * C + (int64_t)splits * d->K;
}

extern "C" int fmd_wgrad(const fmd_wgrad_desc* d, fmd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if ((d->C0 % 8) || (d->C1 % 8) || (d->K % 8) || !d->ws || !d->dw) return -1;
  if (d->ldy > 0 && (d->ldy % 8)) return -3;
  if (d->C1 && !d->src1) return -2;
  WArgs A = make_args(d);
  const int splits = d->splits > 1 ? d->splits : 1;
  int rc = d->force_generic ? 1 : fmd_wgrad_halo(d, stream);
  if (rc == 1) {
    dim3 grid(A.ntc * (A.merged ? A.nci : A.nci * A.T), splits);
    hipLaunchKernelGGL(wgrad_kernel, grid, dim3(256), 0, s, A);
    rc = (int)hipGetLastError();
  }
  if (rc) return rc;
  if (A.T > 27) return -4;
  // one pass: wgrad_reduce2 (all taps per block, slabs over slab lanes); wgrad_reduce when C % 4 != 0.  (Round 3's
  // two-stage form -- groups of 8 slabs summed in place, then wgrad_reduce -- was 0.4 ms per train step slower.)
  if (A.C % 4 == 0) {
    const int sl = max(1, min(splits, 512 / (16 * A.T)));
    hipLaunchKernelGGL(wgrad_reduce2, dim3(d->K, (A.C + RC - 1) / RC), dim3(512), 0, s, A, splits, splits, 1, sl);
  } else {
    hipLaunchKernelGGL(wgrad_reduce, dim3(d->K, (A.C + RC - 1) / RC), dim3(256), 0, s, A, splits, splits, 1);
  }
  return (int)hipGetLastError();
}
