// Halo-tiled 3x3 stride-1 convolution, v11 experiment: ping-pong of two wave groups of ONE workgroup per CU.
//
// Why: v9b runs two independent 256-thread workgroups per CU, one wave of each per SIMD; every wave interleaves its
// MFMAs with its share of the next chunk's GN+SiLU staging and both waves of a SIMD do so at the same time, so the
// staging VALU competes with the MFMA issue of both (PMC: MFMA busy 45 %, ~6 non-MFMA VALU per MFMA).  v10 split
// the roles into producer and consumer waves and lost to the producer's critical path.  v11 alternates the roles:
// one 512-thread workgroup per CU, waves 0-3 (group 0) and 4-7 (group 1) each own one 32-cout quarter of the 16x16 x
// 128-cout tile over half its pixels (4 accumulators of 32x32).  Per chunk, phase A: group 0 runs the chunk's MFMAs
// while group 1 stages its half of the next chunk's halo; phase B: the other way round; a barrier between phases.
// A group's staging loads are issued during its own MFMA phase, the B fragments of a whole chunk (9 taps, 72 VGPRs)
// during its staging phase, so neither waits on memory in the phase that uses them.
//
// Scope of the experiment: 2-D, stride 1, no nearest-x2, no 1x1 segment, no split-K, K % 128 == 0, epilogue = bias +
// optional residual + GroupNorm statistics (the forward's common forms).  Same operand layouts, pre-tiled weights and
// accumulation order per output as v9b (bit-identical outputs).
#include "halo_args.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int NT11 = 512;
constexpr int TH = 16, TW = 16, BCO = 128, BK = 32, KC = BK / 8;
constexpr int WTILE = KC * BCO * 16;
constexpr int CMAX = 512;
constexpr int HROW = TW + 2, HPOS = (TH + 2) * HROW, HPOSP = (HPOS + 7) / 8 * 8;
constexpr int HPAD = (HPOSP + 15) / 16 * 16;
constexpr int HBUF = KC * HPAD * 16;
constexpr int OUT_TILE = TH * TW * BCO * 2;
constexpr int RG = 3;                       // staging rounds per group (group h: rounds 3h .. 3h + 2 of 64 positions)
static_assert(2 * RG * 64 >= HPOSP, "rounds");
constexpr int SM_OUT = 2 * HBUF;
constexpr int SM_COEF = SM_OUT + OUT_TILE;
constexpr int ZCOEF = 2 * CMAX;
constexpr int SM_EPI = SM_COEF + (2 * CMAX + 8) * 4;
constexpr int SM_BYTES = SM_EPI + BCO * 4;
constexpr int DUMMY = (HPOS + 2) * 16;

FMD_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
FMD_DEV bf16x8 as_bf16x8(const u32x4& u) { return __builtin_bit_cast(bf16x8, u); }
FMD_DEV void fence8(float (&y)[8]) {
  asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
}

template <int PRO>
__global__ __launch_bounds__(NT11) void conv3x3_halo11(const HArgs A) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_BYTES];
  float* const coef = (float*)(smem + SM_COEF);
  float* const epi = (float*)(smem + SM_EPI);
  unsigned char* const tileb = smem + SM_OUT;

  const fmd_conv_desc& d = A.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int h = wid >> 2, qd = wid & 3;          // group (pixel half), cout quarter
  const int lt = tid & 255;                      // thread index inside the group
  const int r = lane & 31, hh = lane >> 5, rr = r >> 4;
  const int col = rr ? ((r - 18) & 15) : r;

  const int per_img = A.tiles_x * A.tiles_y;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = b % A.ntc;
  const int tile = b / A.ntc;
  const int n = tile / per_img;
  const int tin = tile - n * per_img;
  const int ty0 = (tin / A.tiles_x) * TH, tx0 = (tin - (tin / A.tiles_x) * A.tiles_x) * TW;
  const int co0 = tco * BCO;
  auto opix = [&](int pi) { return (n * d.Ho + ty0 + (pi >> 4)) * d.Wo + tx0 + (pi & 15); };
  const int hy0 = ty0 - 1, hx0 = tx0 - 1;
  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;

  if (PRO != 0) {
    for (int i = tid; i < 2 * A.C; i += NT11)
      coef[i] = i < A.C ? d.pro_a[(size_t)n * A.C + i] : d.pro_b[(size_t)n * A.C + (i - A.C)];
    if (tid < 8) coef[ZCOEF + tid] = 0.f;
  }
  if (tid < BCO) {
    const int co = co0 + tid;
    float bsum = 0.f;
    if (d.bias) bsum += d.bias[co];
    if (d.bias2) bsum += d.bias2[co];
    if (d.bias_nc) bsum += d.bias_nc[(size_t)n * d.K + co];
    epi[tid] = bsum;
  }
  const int nch = A.nchunk1;

  // ---- B fragments of a whole chunk: tap t -> [plane 4][cout 128][8] bf16 tile, this lane's 2 x 16 bytes
  const unsigned char* const wt1 = (const unsigned char*)(A.wt + (size_t)tco * nch * 9 * (WTILE / 2));
  const int boff = (hh * BCO + 32 * qd + r) * 16;
  bf16x8 bq[9][2];
  auto loadB = [&](int chunk) {
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const unsigned char* base = wt1 + (size_t)(chunk * 9 + t) * WTILE;
      bq[t][0] = *(const bf16x8*)(base + boff);
      bq[t][1] = *(const bf16x8*)(base + boff + 4096);
    }
  };

  // ---- halo staging: this group's rounds 3h .. 3h+2 (64 positions x 4 chunk planes each)
  const int kc = (lt >> 3) & (KC - 1);
  const int p0 = (lt >> 5) * 8 + (lt & 7);
  int spix[RG];
#pragma unroll
  for (int j = 0; j < RG; ++j) {
    const int pos = (RG * h + j) * 64 + p0;
    const int py = pos / HROW, px = pos - (pos / HROW) * HROW;
    const int y = hy0 + py, x = hx0 + px;
    spix[j] = pos >= HPOS ? -2 : (y >= 0 && y < d.Hs && x >= 0 && x < d.Ws) ? y * d.Ws + x : -1;
  }
  const int sdst0 = (kc * HPAD + p0) * 16 + RG * h * 1024;
  const bf16r* sbase = s0;
  int scs = 0, simg = 0, sca = ZCOEF, scb = ZCOEF;
  bool sok = false;
  auto setup = [&](int chunk) {
    const int c = chunk * BK + kc * 8;
    sok = c < A.C;
    sbase = !sok ? s0 : (c < d.C0) ? s0 + c : s1 + (c - d.C0);
    scs = (c < d.C0) ? d.C0 : d.C1;
    simg = n * d.Hs * d.Ws;
    sca = sok ? c : ZCOEF;
    scb = sok ? A.C + c : ZCOEF;
  };
  u32x4 rh[RG];
  auto load_rounds = [&]() {
#pragma unroll
    for (int j = 0; j < RG; ++j) {
      const int sp = spix[j];
      const bf16r* src = (sok && sp >= 0) ? sbase + (size_t)(simg + sp) * scs : s0;
      rh[j] = *(const u32x4*)src;
    }
  };
  auto store_rounds = [&](int buf) {
    float qa[8], qb[8];
    if (PRO != 0) {
      const f32x4 a0 = *(const f32x4*)(coef + sca), a1 = *(const f32x4*)(coef + sca + 4);
      const f32x4 b0 = *(const f32x4*)(coef + scb), b1 = *(const f32x4*)(coef + scb + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) { qa[e] = a0[e]; qa[4 + e] = a1[e]; qb[e] = b0[e]; qb[4 + e] = b1[e]; }
    }
#pragma unroll
    for (int j = 0; j < RG; ++j) {
      const int sp = spix[j];
      const bool valid = sok && sp >= 0;
      const u32x4 raw = rh[j];
      u32x4 v = raw;
      if (PRO != 0) {
        float y[8], t[8];
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          y[2 * e] = bf_lo(raw[e]) * qa[2 * e] + qb[2 * e];
          y[2 * e + 1] = bf_hi(raw[e]) * qa[2 * e + 1] + qb[2 * e + 1];
        }
        if (PRO == 2) {
          fence8(y);
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_exp2f(y[i] * -1.4426950408889634f);
          fence8(t);
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_rcpf(1.f + t[i]);
          fence8(t);
#pragma unroll
          for (int i = 0; i < 8; ++i) y[i] = y[i] * t[i];
        }
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = pack2(y[2 * e], y[2 * e + 1]);
      }
      // padding positions were zeroed once per buffer (their store goes to the dummy slot); invalid channels meet
      // zero coefficients (PRO) or are zeroed here (raw input)
      if (PRO == 0 && !valid) v = u32x4{0u, 0u, 0u, 0u};
      const int dst = sp == -2 ? DUMMY : (sp == -1 ? DUMMY : sdst0 + j * 1024);
      *(u32x4*)(smem + buf + dst) = v;
    }
  };

  // ---- A fragments: this wave's 4 pixel blocks (rows 2pb, 2pb+1 for pb = 4h .. 4h+3), one k-step of a tap
  const int abase = (hh * HPAD + rr * HROW + col) * 16;
  auto aoff = [&](int tap, int s, int pb) {
    const int ky = tap / 3, kx = tap % 3;
    return abase + (s * 2 * HPAD + (2 * pb + ky) * HROW + kx) * 16;
  };
  f32x16 acc[4];
  // a chunk's 9 taps with the A fragments of tap t+1 read while tap t's 8 MFMAs run (one MFMA wave per SIMD in a
  // phase: its own LDS latency must hide under its own MFMAs)
  auto chunk_mma = [&](int hb) {
    bf16x8 af[2][8];
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[0][4 * s + i] = *(const bf16x8*)(smem + hb + aoff(0, s, 4 * h + i));
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) {
#pragma unroll
        for (int s = 0; s < 2; ++s)
#pragma unroll
          for (int i = 0; i < 4; ++i)
            af[(t + 1) & 1][4 * s + i] = *(const bf16x8*)(smem + hb + aoff(t + 1, s, 4 * h + i));
      }
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] = mfma32(af[t & 1][4 * s + i], bq[t][s], acc[i]);
      if (t + 1 < 9) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
          __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        }
      }
    }
  };

  // ---- prologue: padding zeroed in both buffers, chunk 0 staged by both groups, group 1's next-half loads issued
#pragma unroll
  for (int j = 0; j < RG; ++j)
    if (spix[j] == -1) {
      *(u32x4*)(smem + sdst0 + j * 1024) = u32x4{0u, 0u, 0u, 0u};
      *(u32x4*)(smem + HBUF + sdst0 + j * 1024) = u32x4{0u, 0u, 0u, 0u};
    }
  __syncthreads();   // tables
  {
    const float bv = epi[32 * qd + r];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[i][e] = bv;
  }
  loadB(0);
  setup(0);
  load_rounds();
  store_rounds(0);
  if (h == 1 && nch > 1) {
    setup(1);
    load_rounds();
  }
  __syncthreads();

  for (int c = 0; c < nch; ++c) {
    const int hb = (c & 1) * HBUF, nb = ((c + 1) & 1) * HBUF;
    // phase A: group 0 computes chunk c (and issues its loads of chunk c+1); group 1 stores its half of chunk c+1
    if (h == 0) {
      if (c + 1 < nch) {
        setup(c + 1);
        load_rounds();
      }
      chunk_mma(hb);
    } else if (c + 1 < nch) {
      store_rounds(nb);
    }
    __syncthreads();
    // phase B: group 1 computes chunk c (and issues its loads of chunk c+2); group 0 stores its half of chunk c+1;
    // each group's B fragments of chunk c+1 are loaded after its MFMAs of chunk c
    if (h == 1) {
      if (c + 2 < nch) {
        setup(c + 2);
        load_rounds();
      }
      chunk_mma(hb);
      if (c + 1 < nch) loadB(c + 1);
    } else if (c + 1 < nch) {
      store_rounds(nb);
      loadB(c + 1);
    }
    __syncthreads();
  }

  // ---- epilogue (v9b's, over this wave's 4 pixel blocks): residual by identity MFMAs, GroupNorm sums, transpose
  // back to channels-last by permuted-identity MFMAs into the LDS out tile, 16-byte row stores
  const int K = d.K;
  auto pixl = [&](int pb, int pr) {
    const int q = pr >> 4;
    const int cl = q ? ((pr - 18) & 15) : pr;
    return (2 * pb + q) * TW + cl;
  };
  const bool side = d.resid != nullptr;
  const bool stats = d.stats != nullptr;
  bf16x8 inat[2], iperm[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      inat[s][j] = (__bf16)((16 * s + 8 * hh + j) == r ? 1.0f : 0.0f);
      iperm[s][j] = (__bf16)((16 * s + 8 * (j >> 2) + 4 * hh + (j & 3)) == r ? 1.0f : 0.0f);
    }
  const int cl = 32 * qd;
  float st1 = 0.f, st2 = 0.f;
  // side input of pixel block pb: its 32 pixels x 128 couts = 512 16-byte pieces, two per thread of the group,
  // staged into the block's rows of the out tile and read back in the accumulator layout
  auto side_piece = [&](int pb, int j) -> const bf16r* {
    const int qq = lt + 256 * j, pi = 32 * pb + (qq >> 4), c16 = qq & 15;
    return (const bf16r*)d.resid + (size_t)opix(pi) * K + co0 + c16 * 8;
  };
  u32x4 sv[2];
  if (side) {
#pragma unroll
    for (int j = 0; j < 2; ++j) sv[j] = *(const u32x4*)side_piece(4 * h, j);
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const int pb = 4 * h + i;
    const int pi_l = pixl(pb, r);
    f32x16 v = acc[i];
    if (side) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int qq = lt + 256 * j, pi = 32 * pb + (qq >> 4), c16 = qq & 15;
        *(u32x4*)(tileb + pi * 256 + ((c16 ^ (pi & 15)) * 16)) = sv[j];
      }
      __syncthreads();
      if (i + 1 < 4) {
#pragma unroll
        for (int j = 0; j < 2; ++j) sv[j] = *(const u32x4*)side_piece(pb + 1, j);
      }
      bf16x8 fr[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = cl + 16 * s + 8 * hh;
        fr[s] = *(const bf16x8*)(tileb + pi_l * 256 + (((c >> 3) ^ (pi_l & 15)) * 16));
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) v = mfma32(fr[s], inat[s], v);
    }
    bf16x8 pf[2];
#pragma unroll
    for (int s = 0; s < 2; ++s) {
      u32x4 u;
#pragma unroll
      for (int e = 0; e < 4; ++e) u[e] = pack2(v[8 * s + 2 * e], v[8 * s + 2 * e + 1]);
      pf[s] = as_bf16x8(u);
      if (stats) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float w0 = bf_lo(u[e]), w1 = bf_hi(u[e]);
          st1 += w0 + w1;
          st2 += w0 * w0 + w1 * w1;
        }
      }
    }
    f32x16 z;
#pragma unroll
    for (int e = 0; e < 16; ++e) z[e] = 0.f;
#pragma unroll
    for (int s = 0; s < 2; ++s) z = mfma32(pf[s], iperm[s], z);
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int c = cl + 8 * g + 4 * hh;
      u32x2 o;
      o[0] = pack2(z[4 * g], z[4 * g + 1]);
      o[1] = pack2(z[4 * g + 2], z[4 * g + 3]);
      *(u32x2*)(tileb + pi_l * 256 + (((c >> 3) ^ (pi_l & 15)) * 16) + (c & 7) * 2) = o;
    }
    if (stats && (pb & 1)) {   // one statistics row per 64 pixels (pixel blocks 2k, 2k+1)
      const int srow = tile * 4 + (pb >> 1);
      const float a = st1 + __shfl_xor(st1, 32, 64);
      const float q = st2 + __shfl_xor(st2, 32, 64);
      if (hh == 0) {
        float* sp = d.stats + ((size_t)srow * K + co0 + cl + r) * 2;
        sp[0] = a;
        sp[1] = q;
      }
      st1 = 0.f;
      st2 = 0.f;
    }
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < TH * TW * BCO / 8 / NT11; ++k) {
    const int q = tid + NT11 * k, pi = q >> 4, c16 = q & 15;
    *(u32x4*)((bf16r*)d.out + (size_t)opix(pi) * K + co0 + c16 * 8) =
        *(const u32x4*)(tileb + pi * 256 + ((c16 ^ (pi & 15)) * 16));
  }
}

}  // namespace

static int g_halo11 = 0;
// Debug hook (not part of the public ABI): 1 routes the problems v11 supports to it (A/B runs).
extern "C" int fmd_debug_halo11(int on) {
  g_halo11 = on;
  return 0;
}

int halo11_launch(const HArgs& A, int pro, fmd_stream_t stream) {
  const fmd_conv_desc* d = &A.d;
  if (!g_halo11) return 1;
  if (d->upsample || d->Do > 0 || d->Ds > 0 || A.depth || d->src2 || A.nchunk2 || A.splits > 1 || d->gout) return 1;
  if (d->K % BCO || d->out_f32 || d->accumulate || d->ep_x0 || d->ep_a) return 1;
  if (d->pro_a && A.C > CMAX) return 1;
  const int nwg = A.d.N * A.tiles_x * A.tiles_y * A.ntc;
  hipStream_t st = (hipStream_t)stream;
  if (pro == 2) hipLaunchKernelGGL(conv3x3_halo11<2>, dim3(nwg), dim3(NT11), 0, st, A);
  else if (pro == 1) hipLaunchKernelGGL(conv3x3_halo11<1>, dim3(nwg), dim3(NT11), 0, st, A);
  else hipLaunchKernelGGL(conv3x3_halo11<0>, dim3(nwg), dim3(NT11), 0, st, A);
  return (int)hipGetLastError();
}
