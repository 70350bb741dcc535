// Halo-tiled weight gradient for 3x3 stride-1 convolutions (gfx950) -- the UNet's
// dominant backward problem.
//
// dW[co][ci][tap] = sum_p dY[p][co] * G(p + off(tap))[ci], G = SiLU(a*x + b) (the
// forward's fused GroupNorm prologue, recomputed).  A workgroup owns 128 output
// channels x 64 input channels x ALL 9 taps and streams 8x16-pixel tiles of its
// split of the image batch: per tile the 128-pixel dY tile and the 10x18 halo of
// G are staged ONCE into LDS, and every tap reads its shifted pixel rows from the
// same halo image -- 9x less staging/transform work than one workgroup per tap.
// Both operands are pixel-major in HBM, so the reduction (pixel) dimension is the
// strided one: LDS images are chunk-major ([16-byte channel group][position],
// plane stride == 16 banks mod 64) and MFMA fragments come from gfx950's
// transposing ds_read_b64_tr_b16, which is bank-conflict-free on this layout.
// Waves: 2 (64 couts) x 4 (16 cins); each holds 4 x 9 accumulator tiles.
// Tiles are double-buffered: the loads of tile i+1 are in flight while tile i's
// MFMAs run; one barrier per tile.  Partial sums go to a split-K slab reduced by
// wgrad_reduce (csrc/wgrad.hip), which writes the reference [K][C][3][3] layout.
//
// S2D (stride 2): a workgroup's input chunk is one space-to-depth plane (a, b) of the input (pixels (2y + a, 2x + b),
// staged at the output's resolution into the same 10x18 halo) and a 64-channel block; the plane meets only the taps
// ky = 1 (a = 0) or ky in {0, 2} (a = 1) at halo rows {0} / {-1, 0}, columns alike, so the four planes compute the
// 9 taps exactly once between them (1, 2, 2, 4 per plane; the tap loop is instantiated per plane shape).  2-D only:
// on config E's 3-D downsamples the per-plane workgroups (a tile's dY staged once per plane and depth tap, 1-4 taps
// of MFMAs per staging, unequal plane loads) measured slower than the generic kernel.
//
// 3-D (3x3x3): tiles run over the N*D output slices and a workgroup's input chunk is a (depth tap kz,
// 64-channel block) pair staging slice z + kz - 1 (zeros outside the sample, >> 1 under nearest-x2); its
// 9 accumulated taps land at taps kz*9 .. kz*9+8 of a 27-tap slab, so wgrad_reduce writes [K][C][3][3][3].
//
// Replaces: autograd of nn.Conv2d weight/bias (src/nn/ops/convolution.py:53) for
// the ResBlock 3x3 convs (src/nn/blocks/residual.py:71-76).
#include "common.h"
#include "../../include/fmdiff.h"

#ifdef FMD_HALO_DBG
extern int g_dbg;
#define WDBG(bit) (A.dbg & (bit))
#else
#define WDBG(bit) false
#endif

namespace {

constexpr int WTH = 8, WTW = 16;                 // pixel tile
constexpr int WPIX = WTH * WTW;                  // 128 pixels = 4 MFMA k-steps
constexpr int HR = WTW + 2;                      // halo row (18)
constexpr int HPOSW = (WTH + 2) * HR;            // 180 halo positions
constexpr int XPAD = 180;                        // x plane stride in positions (180*4 dwords = 16 mod 64 banks)
constexpr int DPAD = 132;                        // dY plane stride (132*4 = 16 mod 64)
constexpr int WCO = 128, WCI = 64;
constexpr int XPL = WCI / 8, DPL = WCO / 8;      // 16-byte planes
constexpr int XBUF = XPL * XPAD * 8;             // bf16 elements per x buffer
constexpr int DBUF = DPL * DPAD * 8;             // per dY buffer
constexpr int NT = 512;
constexpr int XLD = (HPOSW * XPL + NT - 1) / NT; // x chunks per thread per tile (3)

struct HWArgs {
  fmd_wgrad_desc d;
  int C, ldy;
  int tiles_x, tiles_y, ntiles;    // pixel tiles over N x Ho x Wo
  int ntc, nci, splits, per_split;
  int dbg;                         // ablation flags (FMD_HALO_DBG builds): 1 no G loads, 2 no transform, 4 no dY DMA,
                                   // 8 no MFMA, 16 no per-tile wait + barrier, 32 no slab write
  int depth, ncc, dsrc;            // 3-D (depth > 0): tiles over the N*depth output slices; input chunk
                                   // tci = (depth tap kz, 64-channel block) = kz*ncc + cb reading logical
                                   // slice z + kz - 1 (stored slice >> 1 under nearest-x2; dsrc = stored depth)
};

template <int V> struct IC { static constexpr int value = V; };

// PRO: 0 = raw input, 1 = GroupNorm affine, 2 = affine + SiLU; S2D: stride 2 (planes as chunks)
template <int PRO, bool S2D = false>
__global__ __launch_bounds__(512) void wgrad_halo_kernel(const HWArgs A) {
  __shared__ __attribute__((aligned(16))) bf16r lds[2 * XBUF + 2 * DBUF];
  bf16r* xb = lds;
  bf16r* db_ = lds + 2 * XBUF;
  const unsigned db_base = (unsigned)(size_t)(__attribute__((address_space(3))) bf16r*)db_;
  const fmd_wgrad_desc& d = A.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wco = wid >> 2, wci = wid & 3;
  const int l16 = lane & 15, lq = lane >> 4;
  const int rq = l16 >> 2, rp = lane & 3;          // transposed-read row / column group

  int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tci = b % A.nci; b /= A.nci;
  const int tco = b % A.ntc; b /= A.ntc;
  const int split = b;
  // input chunk: stride 1 tci = kz*ncc + cb (3-D) | cb; S2D (2-D) tci = plane*ncc + cb
  const int cgrp = tci / A.ncc;
  const int pl = S2D ? cgrp : 0, pa_ = pl >> 1, pb_ = pl & 1;
  const int kz = A.depth ? cgrp : 0;   // 3-D: depth tap of this workgroup's input chunk
  const int zsh = A.depth ? kz - 1 : 0;
  const int co0 = tco * WCO, ci0 = (tci - cgrp * A.ncc) * WCI;
  const int T = A.depth ? 27 : 9;
  const int t0 = split * A.per_split, t1 = min(A.ntiles, t0 + A.per_split);
  const bool do_bias = d.db != nullptr && tci == 0;

  const bf16r* __restrict__ dy = (const bf16r*)d.dy;
  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;

  // this thread's staging slots: x channel group kx8 (fixed) at halo positions (tid & 7) + 8 * (tid >> 6) + 64 k,
  // so the 8-lane groups of ds_write_b128 store 8 consecutive positions of one plane (32 distinct banks)
  const int kx8 = (tid >> 3) & 7;
  const int c = ci0 + kx8 * 8;
  const bf16r* xsrc = (c < d.C0) ? s0 + c : s1 + (c - d.C0);
  const int xcs = (c < d.C0) ? d.C0 : d.C1;
  float pa[8], pb[8];

  auto tile_org = [&](int t, int& n, int& ty0, int& tx0) {
    const int per_img = A.tiles_x * A.tiles_y;
    n = t / per_img;
    const int r = t - n * per_img;
    ty0 = (r / A.tiles_x) * WTH;
    tx0 = (r - (r / A.tiles_x) * A.tiles_x) * WTW;
  };

  u32x4 rx[XLD];
  int xo[XLD];                  // LDS offset, -1 none, bit 30 zero padding
  int cur_n = -1;

  auto load_tile = [&](int t) {
    int n, ty0, tx0;
    tile_org(t, n, ty0, tx0);
    const int smp = A.depth ? n / A.depth : n;   // sample of image n (3-D: slices share the affine)
    if (PRO != 0 && smp != cur_n) {   // GN affine of this thread's 8 channels for sample smp
      const f32x4* a4 = (const f32x4*)(d.pro_a + (size_t)smp * A.C + c);
      const f32x4* b4 = (const f32x4*)(d.pro_b + (size_t)smp * A.C + c);
      const f32x4 a0 = a4[0], a1 = a4[1], b0 = b4[0], b1 = b4[1];
#pragma unroll
      for (int e = 0; e < 4; ++e) { pa[e] = a0[e]; pa[4 + e] = a1[e]; pb[e] = b0[e]; pb[4 + e] = b1[e]; }
      cur_n = smp;
    }
    const int zl = A.depth ? n - smp * A.depth + zsh : 0;   // logical input slice (== output depth range)
    const bool zok = !A.depth || (zl >= 0 && zl < A.depth);
    const int srcsl = A.depth ? smp * A.dsrc + (d.upsample ? zl >> 1 : zl) : n;
#pragma unroll
    for (int k = 0; k < XLD; ++k) {
      const int pos = (tid & 7) + 8 * (tid >> 6) + (NT / 8) * k;
      const bool act = pos < HPOSW;
      const int hy = act ? pos / HR : 0, hx = act ? pos - (pos / HR) * HR : 0;
      // logical (possibly nearest-x2-upsampled) input coordinates; the upsample is a gather of the
      // stored low-resolution pixel, so the LDS image is the same as without it
      const int y = ty0 - 1 + hy, x = tx0 - 1 + hx;
      const bool valid = act && zok && y >= 0 && y < d.Ho && x >= 0 && x < d.Wo;
      const int sy = S2D ? 2 * y + pa_ : d.upsample ? y >> 1 : y, sx = S2D ? 2 * x + pb_ : d.upsample ? x >> 1 : x;
      const int pix = valid ? (srcsl * d.Hs + sy) * d.Ws + sx : 0;
      rx[k] = WDBG(1) ? u32x4{0u, 0u, 0u, 0u} : *(const u32x4*)(xsrc + (size_t)pix * xcs);
      xo[k] = !act ? -1 : ((kx8 * XPAD + pos) * 8) | (valid ? 0 : (1 << 30));
    }
  };
  // dY needs no transform: gathered global -> LDS by DMA (lane = one pixel's 16-byte channel group).
  // Issued through inline asm (glds16): the builtin form makes hipcc drain vmcnt before every later
  // LDS read, i.e. the next tile's loads would be waited for inside this tile's MFMA loop.
  auto dma_dy = [&](int t, int buf) {
    int n, ty0, tx0;
    tile_org(t, n, ty0, tx0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int idx = wid * 4 + j, plane = idx >> 1, half = idx & 1;
      const int pos = half * 64 + lane;
      const int pix = (n * d.Ho + ty0 + (pos >> 4)) * d.Wo + tx0 + (pos & 15);
      const unsigned dst = db_base + (unsigned)(buf * DBUF + (plane * DPAD + half * 64) * 8) * 2;
      if (!WDBG(4)) glds16(dy + (size_t)pix * A.ldy + co0 + plane * 8, __builtin_amdgcn_readfirstlane(dst));
    }
  };
  auto store_tile = [&](int buf) {
#pragma unroll
    for (int k = 0; k < XLD; ++k) {
      u32x4 v = rx[k];
      if (PRO != 0 && !WDBG(2)) {
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float lo = bf_lo(v[e]) * pa[2 * e] + pb[2 * e];
          float hi = bf_hi(v[e]) * pa[2 * e + 1] + pb[2 * e + 1];
          if (PRO == 2) { lo = siluf_(lo); hi = siluf_(hi); }
          v[e] = pack2(lo, hi);
        }
      }
      const int o = xo[k];
      if (o & (1 << 30)) v = u32x4{0u, 0u, 0u, 0u};
      if (o >= 0) *(u32x4*)(xb + buf * XBUF + (o & ~(1 << 30))) = v;
    }
  };

  f32x4 acc[4][9];
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int t = 0; t < 9; ++t) acc[i][t] = f32x4{0.f, 0.f, 0.f, 0.f};

  float dbs[4] = {0.f, 0.f, 0.f, 0.f};   // bias partials of this lane's 4 couts (from the A fragments)

  // one pixel tile: 4 k-steps (32 pixels each) x 9 taps x 4 cout blocks = 144 MFMAs.  Fully unrolled and
  // software-pipelined: the B fragment (G at the tap's shifted pixels) of tap slot s + 2 is read at slot s (a
  // 3-deep ring) and the next k-step's A fragments (dY^T) half-way through a k-step, so no MFMA waits on the LDS
  // read it consumes (round 3: read -> wait -> 4 MFMAs per tap)
  const bf16r* const abase = db_ + ((wco * 8 + (rp >> 1)) * DPAD + (lq >> 1) * WTW + 8 * (lq & 1) + rq) * 8 + (rp & 1) * 4;
  const bf16r* const bbase = xb + ((wci * 2 + (rp >> 1)) * XPAD + (lq >> 1) * HR + 8 * (lq & 1) + rq) * 8 + (rp & 1) * 4;
  auto readA = [&](int buf, int ks, bf16x8 (&a)[4]) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const bf16r* p = abase + buf * DBUF + (ks * 2 * WTW + 2 * i * DPAD) * 8;
      const s16x4 lo = ds_read_tr16(p), hi = ds_read_tr16(p + 4 * 8);
      a[i] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    }
  };
  auto compute = [&](int buf) {
    bf16x8 af[2][4], bq[3];
    auto readB = [&](int sl) {
      const int ks = sl / 9, tap = sl % 9, ky = tap / 3, kx = tap % 3;
      const bf16r* p = bbase + buf * XBUF + ((2 * ks + ky) * HR + kx) * 8;
      const s16x4 lo = ds_read_tr16(p), hi = ds_read_tr16(p + 4 * 8);
      bq[sl % 3] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    readA(buf, 0, af[0]);
    readB(0);
    readB(1);
#pragma unroll
    for (int sl = 0; sl < 36; ++sl) {
      const int ks = sl / 9, tap = sl % 9;
      if (tap == 4 && ks < 3) readA(buf, ks + 1, af[(ks + 1) & 1]);
      if (sl + 2 < 36) readB(sl + 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][tap] = mfma16(af[ks & 1][i], bq[sl % 3], acc[i][tap]);
    }
  };
  // S2D: the plane's NTY x NTX taps at halo rows hy0 + jy, columns hx0 + jx (accumulator slot jy * NTX + jx)
  const int hy0 = pa_ ? 0 : 1, hx0 = pb_ ? 0 : 1;
  auto compute_s2d = [&](int buf, auto nty, auto ntx) {
    constexpr int NTY = decltype(nty)::value, NTX = decltype(ntx)::value, NTP = NTY * NTX, NS = 4 * NTP;
    bf16x8 af[2][4], bq[3];
    auto readB = [&](int sl) {
      const int ks = sl / NTP, t = sl % NTP, jy = t / NTX, jx = t % NTX;
      const bf16r* p = bbase + buf * XBUF + ((2 * ks + hy0 + jy) * HR + hx0 + jx) * 8;
      const s16x4 lo = ds_read_tr16(p), hi = ds_read_tr16(p + 4 * 8);
      bq[sl % 3] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
    };
    readA(buf, 0, af[0]);
    readB(0);
    if (NS > 1) readB(1);
#pragma unroll
    for (int sl = 0; sl < NS; ++sl) {
      const int ks = sl / NTP, t = sl % NTP;
      if (t == NTP / 2 && ks < 3) readA(buf, ks + 1, af[(ks + 1) & 1]);
      if (sl + 2 < NS) readB(sl + 2);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][t] = mfma16(af[ks & 1][i], bq[sl % 3], acc[i][t]);
    }
  };
  // bias partials (workgroups of the first cin block): each wave sums k-step wci's 32 pixels of its 64 couts, so
  // the four cin waves of a cout half cover the tile
  auto bias_sums = [&](int buf) {
    bf16x8 a[4];
    readA(buf, wci, a);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      float sacc = 0.f;
#pragma unroll
      for (int e = 0; e < 8; ++e) sacc += (float)a[i][e];
      dbs[i] += sacc;
    }
  };

  if (t0 < t1) {
    dma_dy(t0, 0);
    load_tile(t0);
    store_tile(0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the asm DMAs are not tracked by hipcc
    __syncthreads();
    int buf = 0;
    for (int t = t0; t < t1; ++t) {
      const bool more = t + 1 < t1;
      if (more) {
        load_tile(t + 1);
        dma_dy(t + 1, buf ^ 1);
      }
      if (!WDBG(8)) {
        if (!S2D) compute(buf);
        else if (pl == 0) compute_s2d(buf, IC<1>(), IC<1>());
        else if (pl == 1) compute_s2d(buf, IC<1>(), IC<2>());
        else if (pl == 2) compute_s2d(buf, IC<2>(), IC<1>());
        else compute_s2d(buf, IC<2>(), IC<2>());
      }
      if (do_bias) bias_sums(buf);
      if (more) store_tile(buf ^ 1);
      if (!WDBG(16)) {
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // next tile's dY DMA landed before the barrier
        __syncthreads();
      }
      buf ^= 1;
    }
  }

  if (WDBG(32)) return;
  // ---- partial slab ws[split][co][tap][ci] (wgrad_reduce's layout; 3-D tap = kz*9 + ky*3 + kx)
  const size_t per = (size_t)d.K * T * A.C;
  float* ws = d.ws + (size_t)split * per;
  // S2D: slot jy * NTX + jx of plane (a, b) is tap (ky, kx) = (a ? 2 jy : 1, b ? 2 jx : 1)
  const int ntx = pb_ ? 2 : 1, nts = (pa_ ? 2 : 1) * ntx;
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int slot = 0; slot < (S2D ? 4 : 9); ++slot) {
      if (S2D && slot >= nts) continue;
      const int jy = slot / ntx, jx = slot - jy * ntx;
      const int tap = !S2D ? slot : (pa_ ? 2 * jy : 1) * 3 + (pb_ ? 2 * jx : 1);
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int co = co0 + wco * 64 + 16 * i + 4 * lq + r;
        const int ci = ci0 + wci * 16 + l16;
        ws[((size_t)co * T + kz * 9 + tap) * A.C + ci] = acc[i][slot][r];
      }
    }
  if (do_bias) {
    // lanes of the 4 pixel groups, then the 4 cin-waves (each summed one k-step) of a cout half
    float* red = (float*)lds;    // [4 wci][128 co] floats; the tiles are done
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      dbs[i] += __shfl_xor(dbs[i], 16, 64);
      dbs[i] += __shfl_xor(dbs[i], 32, 64);
    }
    __syncthreads();
    if (lq == 0) {
#pragma unroll
      for (int i = 0; i < 4; ++i) red[wci * WCO + wco * 64 + 16 * i + l16] = dbs[i];
    }
    __syncthreads();
    if (tid < WCO) {
      const float v = red[tid] + red[WCO + tid] + red[2 * WCO + tid] + red[3 * WCO + tid];
      d.ws[(size_t)A.splits * per + (size_t)split * d.K + co0 + tid] = v;
    }
  }
}

}  // namespace

// 3x3 / stride 1 / pad 1 (optionally on the nearest-x2 upsample of src) or 2-D stride 2 / pad 1 (Hs = 2 Ho,
// Ws = 2 Wo), K % 128 == 0, C % 64 == 0, Ho % 8 == 0, Wo % 16 == 0.
// Returns 1 (nothing launched) when the problem does not qualify.  d->splits = pixel-tile splits.
extern "C" int fmd_wgrad_halo(const fmd_wgrad_desc* d, fmd_stream_t stream) {
  const bool s2 = d->stride == 2;   // S2D (2-D): the input's space-to-depth planes as chunks
  if (d->ks != 3 || (d->stride != 1 && !s2) || d->pad != 1 || (s2 && d->upsample)) return 1;
  const bool d3 = d->Do > 0 || d->Ds > 0;
  if (d3 && (s2 || d->Do != (d->upsample ? 2 * d->Ds : d->Ds))) return 1;   // 3-D: stride-1 3x3x3 (nearest-x2)
  const int Nn = d3 ? d->N * d->Do : d->N;                // images (3-D: depth slices)
  if (s2 ? (d->Hs != 2 * d->Ho || d->Ws != 2 * d->Wo)
         : d->upsample ? (d->Ho != 2 * d->Hs || d->Wo != 2 * d->Ws) : (d->Ho != d->Hs || d->Wo != d->Ws)) return 1;
  if (d->Ho % WTH || d->Wo % WTW) return 1;
  const int C = d->C0 + d->C1;
  if (d->K % WCO || C % WCI || (d->C0 % 8) || !d->ws) return 1;
  const int ldy = d->ldy > 0 ? d->ldy : d->K;
  if (ldy % 8) return 1;
  if ((long long)Nn * d->Hs * d->Ws >= (1LL << 31) / 8) return 1;
  HWArgs A;
  A.d = *d;
  A.C = C;
  A.ldy = ldy;
  A.tiles_x = d->Wo / WTW;
  A.tiles_y = d->Ho / WTH;
  A.ntiles = Nn * A.tiles_x * A.tiles_y;
  A.ntc = d->K / WCO;
  A.depth = d3 ? d->Do : 0;
  A.dsrc = d3 ? d->Ds : 0;
  A.ncc = C / WCI;
  A.nci = (d3 ? 3 : s2 ? 4 : 1) * A.ncc;
  A.splits = d->splits > 1 ? d->splits : 1;
  A.per_split = (A.ntiles + A.splits - 1) / A.splits;
#ifdef FMD_HALO_DBG
  A.dbg = g_dbg;
#else
  A.dbg = 0;
#endif
  const int nwg = A.ntc * A.nci * A.splits;
  const int pro = d->pro_a ? (d->pro_silu ? 2 : 1) : 0;
  hipStream_t st = (hipStream_t)stream;
  if (s2) {
    if (pro == 2) hipLaunchKernelGGL((wgrad_halo_kernel<2, true>), dim3(nwg), dim3(NT), 0, st, A);
    else if (pro == 1) hipLaunchKernelGGL((wgrad_halo_kernel<1, true>), dim3(nwg), dim3(NT), 0, st, A);
    else hipLaunchKernelGGL((wgrad_halo_kernel<0, true>), dim3(nwg), dim3(NT), 0, st, A);
  } else if (pro == 2) hipLaunchKernelGGL(wgrad_halo_kernel<2>, dim3(nwg), dim3(NT), 0, st, A);
  else if (pro == 1) hipLaunchKernelGGL(wgrad_halo_kernel<1>, dim3(nwg), dim3(NT), 0, st, A);
  else hipLaunchKernelGGL(wgrad_halo_kernel<0>, dim3(nwg), dim3(NT), 0, st, A);
  return (int)hipGetLastError();
}
