// Halo-tiled 3x3 stride-1 convolution (v9b): the UNet's dominant problem on v_mfma_f32_32x32x16_bf16.
//
// Same tiling contract as conv_halo.hip (16x16-pixel x 128-output-channel tile, 32-channel reduction chunks whose
// 18x18 halo -- 10x10 under nearest-x2 -- is staged ONCE into LDS with the GroupNorm affine + SiLU applied, two
// halo buffers), re-budgeted for registers:
//
// * 256-thread workgroups (4 waves, 2 per CU: one wave of each workgroup per SIMD) at up to 256 VGPRs; a wave owns
//   one 32-cout quarter of the tile over all 256 pixels (8 accumulators of 32x32).
// * MFMA 32x32x16: A = activations (rows = 32 pixels = two tile rows, k = 16 channels), B = weights (k = 16
//   channels, cols = 32 couts), B fragments straight from L2 (pre-tiled weights, one tap's 32 x 32 slice per wave).
// * The 9 taps of a chunk are unrolled at compile time: every fragment read is one ds_read_b128 from a fixed base
//   VGPR with an immediate offset.  Halo of the next chunk: rounds of one 16-byte piece per thread, each loaded
//   FMD_H9_LAG taps before it is transformed and stored.
// * A-fragment pixel map: lanes 0-15 read row 2b of the tile, lanes 16-31 row 2b+1 shifted by 2 columns
//   (sigma(x) = (x - 2) mod 16), which makes every ds_read_b128 lane group of gfx950 touch 16 distinct bank slots.
// * Epilogue in the accumulator layout (pixels in registers, couts on lanes): bias as the accumulators' start value,
//   the residual and the data-gradient side input brought into that layout by two MFMAs against an identity
//   (exact), per-channel GroupNorm sums in-lane (+ one cross-half add), and the output transposed back to
//   channels-last by two more MFMAs against a permuted identity, staged in LDS and stored as 16-byte rows.
// (The round-4 v9 variants with an LDS weight ring were measured slower and removed in round 5.)
#include "halo_args.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

constexpr int NT9 = 256;
constexpr int TH = 16, TW = 16, BCO = 128, BK = 32, KC = BK / 8;
constexpr int WTILE = KC * BCO * 16;   // bytes of one tap's weight tile (8 KiB)
constexpr int CMAX = 512;              // widest GN-prologue input of the affine table
constexpr int OUT_TILE = TH * TW * BCO * 2;
constexpr int ZFLAG = 1 << 30;         // staged-piece flag: store zeros (padding)
#ifndef FMD_H9_SCHED
#define FMD_H9_SCHED 1
#endif
constexpr bool H9_SCHED = FMD_H9_SCHED;   // v9b: pinned read/MFMA interleave of a tap (build flag for A/B)
#ifndef FMD_H9_LAG
#define FMD_H9_LAG 3   // taps between a staging round's load and its transform (2: 22.94 / 23.00 vs 3: 22.89 / 22.89 ms per train step)
#endif

template <bool UP, int THT = TH>
struct G9 {
  static constexpr int HROW = UP ? TW / 2 + 2 : TW + 2;           // halo row (positions)
  static constexpr int HPOS = UP ? (THT / 2 + 2) * HROW : (THT + 2) * HROW;
  static constexpr int HPOSP = (HPOS + 7) / 8 * 8;                 // positions rounded to 8-position pieces rows
  static constexpr int HPAD = (HPOSP + 15) / 16 * 16;              // plane stride == 0 mod 16 bank slots
  static constexpr int HBUF = KC * HPAD * 16;                      // bytes per halo buffer
  static constexpr int NPIECE = HPOSP * KC;
  static constexpr int NR = (NPIECE + NT9 - 1) / NT9;              // staging rounds per chunk (6 | 2)
  static_assert(NR <= 6 && NR * NT9 >= NPIECE, "staging rounds");
};

FMD_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

FMD_DEV bf16x8 as_bf16x8(const u32x4& u) { return __builtin_bit_cast(bf16x8, u); }
#ifndef FMD_H9_FENCE
#define FMD_H9_FENCE 1   // staging transform advanced stage by stage behind register fences: fwd 164.5 / 163.0 ->
                         // 159.9 / 161.0 us (8x256^2x128, interleaved A/B, round 5), bit-identical outputs
#endif
FMD_DEV void fence8_(float (&y)[8]) {
  asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
}

// debug ablations (A.dbg via fmd_debug_halo_flags; compiled in only with -DFMD_HALO_DBG, tools/build_variant.sh):
// 1 no halo loads, 2 no transform, 4 no epilogue, 8 no weight DMA in the loop, 128 no step barrier, 256 no MFMA
#ifdef FMD_HALO_DBG
#define HDBG9(bit) (A.dbg & (bit))
#else
#define HDBG9(bit) false
#endif

// ---------------------------------------------------------------------------------------------------------------
// v9b: the same tile, staging and epilogue, with the weights taken straight from L2 into registers.
//
// Each wave owns one 32-cout quarter of the tile over all 256 pixels (8 pixel blocks of 2 rows = 8 accumulators);
// its B fragments (32 couts x 32 channels of one tap, 2 KiB) are two 16-byte global loads per lane, issued one tap
// ahead.  No LDS weight ring means no per-tap DMA and no per-tap barrier: the only workgroup barrier is at the chunk
// boundary (the staged halo of the next chunk complete, the previous buffer free), so the four waves and the two
// workgroups of a CU run their 9 taps independently.  Every load is an ordinary one, so hipcc counts all waits.
//
// S2D: a stride-2 pad-1 conv (3x3, or the 4x4 that folds a nearest-x2 upsample into its data gradient) as a stride-1
// 2x2 conv over the space-to-depth view of its input: plane (a, b) = the pixels (2y + a, 2x + b) at the output's
// resolution, staged straight from the full-resolution NHWC tensor (chunk = plane-major 32-channel block); each
// plane meets the taps u = 1 + 2i (a = 0) or 2i (a = 1), i.e. halo rows {0, +1} or {-1, 0} around the output row
// (columns alike), 4 taps per chunk.  For the 3x3 the a = 0 row / b = 0 column taps at +1 carry zero weights
// (16 tap-planes for 9 taps).  Weights pre-tiled as a 2x2 conv over 4C channels (fmd_s2d_tile_weights).
//
// D2S: the data gradient of a stride-2 3x3 conv (transposed gather) as a stride-1 2x2 conv from the low-resolution
// gradient onto the depth-to-space view of the output: output class (a, b) = the pixels (2i + a, 2j + b), each a
// block of 4 x cout "channels" (class-major, one class per 128-cout tile), meeting dy at offsets {0, +1} (taps
// 1 | 2, 0 per dimension; 9 of the 16 tap-classes non-zero); the epilogue writes the class's pixels.
// MODE: 0 plain 3x3, 1 S2D, 2 D2S.
//
// 3-D (A.depth > 0) stride-2 modes: depth is handled by chunks, in-plane as above.  S2D: images are the N*Do output
// slices and chunk = (depth tap kz < ks, plane, block) stages full-resolution slice 2z + kz - 1 (zeros outside the
// sample).  D2S: images are the N*Ds gradient slices, the output classes are 8 (depth parity, a, b; class-major) and
// chunk = (depth offset dz, block) stages gradient slice z + dz; class (c, a, b) writes full-resolution slice 2z + c.
// THT: tile rows (16, or 8 for grids that would otherwise leave CUs with one workgroup or one round: twice the
// workgroups, half the accumulators)
template <bool UP, int PRO, int MODE = 0, int THT = TH>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(2, 2)))
void conv3x3_halo9b(const HArgs A) {
  static_assert(THT == TH || THT == 8 || THT == 4, "16-, 8- or 4-row tiles");
  using G = G9<UP, THT>;
  constexpr int NPB = THT / 2;               // 32-pixel blocks (2 rows) per wave
  constexpr int OUT_T = THT * TW * BCO * 2;
  constexpr int HROW = G::HROW, HPAD = G::HPAD, HBUF = G::HBUF, NR = G::NR;
  constexpr bool S2D = MODE == 1, D2S = MODE == 2;
  static_assert(!(MODE && UP), "stride-2 modes are not nearest-x2 gathers");
  constexpr int NTAP = MODE ? 4 : 9;         // taps per chunk
  constexpr int RPT = MODE ? 2 : 1;          // staging rounds loaded per tap
  constexpr int LAG = MODE ? 1 : FMD_H9_LAG;  // taps between a round's load and its transform + store
  constexpr int SL = RPT * LAG;              // staging register slots (rounds in flight)
  constexpr int RB = MODE ? 4 : 3;           // B-fragment ring (NTAP % RB == 0 keeps its phase per chunk)
  static_assert(NTAP % RB == 0 && (NR + RPT - 1) / RPT + LAG <= NTAP, "chunk pipeline");
  constexpr int SM_COEF = 2 * HBUF > OUT_T ? 2 * HBUF : OUT_T;
  constexpr int ZCOEF = 2 * CMAX;   // 8 zero coefficients: the affine of a chunk's invalid channels (-> SiLU(0) = 0)
  constexpr int SM_EPI = SM_COEF + (2 * CMAX + 8) * 4;
  constexpr int SM_BYTES = SM_EPI + 3 * BCO * 4;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_BYTES];
  float* const coef = (float*)(smem + SM_COEF);
  float* const epi = (float*)(smem + SM_EPI);

  const fmd_conv_desc& d = A.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;   // wave = 32-cout quarter of the tile
  const int r = lane & 31, hh = lane >> 5, rr = r >> 4;
  const int col = rr ? ((r - 18) & 15) : r;

  const int per_img = A.tiles_x * A.tiles_y;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = b % A.ntc;
  const int tile = b / A.ntc;
  const int n = tile / per_img;
  const int tin = tile - n * per_img;
  const int smp = A.depth ? n / A.depth : n;
  const int zz = A.depth ? n - smp * A.depth : 0;
  const int ty0 = (tin / A.tiles_x) * THT, tx0 = (tin - (tin / A.tiles_x) * A.tiles_x) * TW;
  // D2S: cout tile tco = (output class, 128-cout block), class-major
  const int ncob = D2S ? d.K / BCO : 1;
  const int ocls = D2S ? tco / ncob : 0;
  const int co0 = (D2S ? tco - ocls * ncob : tco) * BCO;
  // output pixel of tile-local pixel pi (y * 16 + x); D2S: the class's full-resolution pixel
  auto opix = [&](int pi) -> int {
    const int y = ty0 + (pi >> 4), x = tx0 + (pi & 15);
    if (D2S) {
      const int no = A.depth ? smp * d.Do + 2 * zz + (ocls >> 2) : n;
      return (no * d.Ho + 2 * y + ((ocls >> 1) & 1)) * d.Wo + 2 * x + (ocls & 1);
    }
    return (n * d.Ho + y) * d.Wo + x;
  };
  const int hy0 = UP ? (ty0 >> 1) - 1 : ty0 - 1;
  const int hx0 = UP ? (tx0 >> 1) - 1 : tx0 - 1;
  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;
  const bf16r* __restrict__ s2 = (const bf16r*)d.src2;
  const bf16r* __restrict__ s3 = (const bf16r*)d.src3;

  if (PRO != 0 && d.fold_st0) {
    // The GroupNorm affine of the sample folded here from the producers' statistics slabs (forward only).  Channel
    // totals: per source its sample's E slab rows x Cx channels are contiguous; thread u of (channel pair, row group)
    // sums rows rg, rg + R, ... as 16-byte loads eight in flight, the R row groups meet in LDS (staging area, not in
    // use yet) in fixed order.  Then per channel the group sums in fp64 (E[x^2] - mean^2, as gn_prep; rstd by the
    // fp32 rsqrt), the affine and the scale-shift rows.
    float2* tot = (float2*)smem;                       // [C] (sum, sum of squares)
    f32x4* prt = (f32x4*)(smem + CMAX * 8);            // [R][pairs] partials
    {
      // both sources in one pass: pair index pi < P0 is src0's, the rest src1's
      const int P0 = d.C0 >> 1, P = A.C >> 1, R = P >= NT9 ? 1 : NT9 / P;
      for (int u = tid; u < P * R; u += NT9) {
        const int rg = u / P, pi = u - rg * P;
        const bool in0 = pi < P0;
        const int pairs = in0 ? P0 : P - P0, pr = in0 ? pi : pi - P0, E = in0 ? A.fold_E0 : A.fold_E1;
        const f32x4* base = (const f32x4*)(in0 ? d.fold_st0 : d.fold_st1) + (size_t)smp * E * pairs + pr;
        f32x4 acc[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
        int e = rg;
        for (; e + 7 * R < E; e += 8 * R) {
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[j] += base[(size_t)(e + j * R) * pairs];
        }
        for (; e < E; e += R) acc[0] += base[(size_t)e * pairs];
        prt[u] = ((acc[0] + acc[1]) + (acc[2] + acc[3])) + ((acc[4] + acc[5]) + (acc[6] + acc[7]));
      }
      __syncthreads();
      for (int pi = tid; pi < P; pi += NT9) {
        f32x4 t = prt[pi];
        for (int rg = 1; rg < R; ++rg) t += prt[rg * P + pi];
        tot[2 * pi] = make_float2(t[0], t[1]);
        tot[2 * pi + 1] = make_float2(t[2], t[3]);
      }
      __syncthreads();
    }
    const int Cg = A.C / d.fold_G;
    for (int c = tid; c < A.C; c += NT9) {
      const int g0 = c - c % Cg;
      double t1 = 0.0, t2 = 0.0;
      for (int j = 0; j < Cg; ++j) {
        const float2 t = tot[g0 + j];
        t1 += t.x;
        t2 += t.y;
      }
      const double mean = t1 * A.fold_inv;
      double var = t2 * A.fold_inv - mean * mean;
      if (var < 0) var = 0;
      const float rs = rsqrtf((float)var + d.fold_eps);
      float a = rs * (d.fold_gamma ? d.fold_gamma[c] : 1.f);
      float bb = (d.fold_beta ? d.fold_beta[c] : 0.f) - (float)mean * a;
      if (d.fold_emb) {
        const float sc = 1.f + d.fold_emb[(size_t)smp * d.fold_emb_stride + c];
        a *= sc;
        bb = bb * sc + d.fold_emb[(size_t)smp * d.fold_emb_stride + A.C + c];
      }
      coef[c] = a;
      coef[A.C + c] = bb;
    }
    if (tid < 8) coef[ZCOEF + tid] = 0.f;
    __syncthreads();   // the staging area is free again
  } else if (PRO != 0) {
    for (int i = tid; i < 2 * A.C; i += NT9)
      coef[i] = i < A.C ? d.pro_a[(size_t)smp * A.C + i] : d.pro_b[(size_t)smp * A.C + (i - A.C)];
    if (tid < 8) coef[ZCOEF + tid] = 0.f;
  }
  if (tid < BCO) {
    const int co = co0 + tid;
    const bool ok = co < d.K;
    float bsum = 0.f;
    if (ok && d.bias) bsum += d.bias[co];
    if (ok && d.bias2) bsum += d.bias2[co];
    if (ok && d.bias_nc) bsum += d.bias_nc[(size_t)smp * d.K + co];
    epi[tid] = bsum;
    epi[BCO + tid] = (ok && d.ep_a) ? d.ep_a[(size_t)smp * d.K + co] : 0.f;
    epi[2 * BCO + tid] = (ok && d.ep_b) ? d.ep_b[(size_t)smp * d.K + co] : 0.f;
  }

  const int split = blockIdx.y;
  const int c_lo = split * A.cps, c_hi = min(A.nchunk1, c_lo + A.cps);
  const int n_seg2 = split == A.splits - 1 ? A.nchunk2 : 0;
  const int T1 = A.nchunk1 * NTAP;

  // ---- B fragments from global: slot sl (tap of the whole reduction) -> [plane 4][cout 128][8] bf16 tile
  const unsigned char* const wt1 = (const unsigned char*)(A.wt + (size_t)tco * T1 * (WTILE / 2));
  const unsigned char* const wt2b = (const unsigned char*)(A.wt2 + (size_t)tco * A.nchunk2 * (WTILE / 2));
  const int boff = (hh * BCO + 32 * wid + r) * 16;   // this lane's 16 bytes of k-step 0 (k-step 1: + 4096)
  auto loadB = [&](bf16x8 (&bq)[2], int sl) {
    const unsigned char* base = sl < T1 ? wt1 + (size_t)sl * WTILE : wt2b + (size_t)(sl - T1) * WTILE;
    bq[0] = *(const bf16x8*)(base + boff);
    bq[1] = *(const bf16x8*)(base + boff + 4096);
  };

  // ---- halo staging (as v9)
  const int kc = (tid >> 3) & (KC - 1);
  const int p0 = (tid >> 5) * 8 + (tid & 7);
  int spix[NR];
#pragma unroll
  for (int q = 0; q < NR; ++q) {
    const int pos = q * 64 + p0;
    const int py = pos / HROW, px = pos - (pos / HROW) * HROW;
    const int y = hy0 + py, x = hx0 + px;
    if (S2D)   // full-resolution pixel (2y, 2x) of the output-resolution halo position; + the plane's (a, b) per chunk
      spix[q] = pos >= G::HPOS ? -2 : (y >= 0 && y < d.Ho && x >= 0 && x < d.Wo) ? 2 * y * d.Ws + 2 * x : -1;
    else
      spix[q] = pos >= G::HPOS ? -2 : (y >= 0 && y < d.Hs && x >= 0 && x < d.Ws) ? y * d.Ws + x : -1;
  }
  const int sdst0 = (kc * HPAD + p0) * 16;
  const int s2pix0 = (n * d.Ho + ty0 + (p0 >> 4)) * d.Wo + tx0 + (p0 & 15);
  const int s2dst0 = (kc * HPAD + ((p0 >> 4) + 1) * (TW + 2) + (p0 & 15) + 1) * 16;
  const int HWs = d.Hs * d.Ws;
  constexpr int DUMMY = (G::HPOS + 2) * 16;
  const bf16r* sbase = s0;
  int scs = 0, simg = 0, sca = 0, scb = 0;
  bool sok = false, sseg2 = false;
  auto setup = [&](int chunk) {
    sseg2 = chunk >= A.nchunk1;
    if (chunk < 0) {
      sok = false; sbase = s0; scs = 0; simg = 0; sca = ZCOEF; scb = ZCOEF;
    } else if (!sseg2) {
      int cb = chunk;
      bool zok = true;
      int sl = n;
      int poff = 0;
      if (S2D) {
        int ch = chunk;
        if (A.depth) {   // 3-D: depth tap kz of a (kz, plane, block) chunk
          const int kz = ch / (4 * A.ncb);
          ch -= kz * 4 * A.ncb;
          const int zl = 2 * zz + kz - 1;
          zok = zl >= 0 && zl < A.dsrc;
          sl = smp * A.dsrc + zl;
        }
        const int pl = ch / A.ncb;   // plane (a, b) = (pl >> 1, pl & 1)
        cb = ch - pl * A.ncb;
        poff = (pl >> 1) * d.Ws + (pl & 1);
      } else if (D2S && A.depth) {   // 3-D: depth offset dz of a (dz, block) chunk
        const int dz = chunk / A.ncb;
        cb = chunk - dz * A.ncb;
        zok = zz + dz < A.dsrc;
        sl = smp * A.dsrc + zz + dz;
      } else if (A.depth) {
        const int kz = chunk / A.ncb;
        cb = chunk - kz * A.ncb;
        const int zl = zz + kz - 1;
        zok = zl >= 0 && zl < A.depth;
        sl = smp * A.dsrc + (UP ? zl >> 1 : zl);
      }
      const int c = cb * BK + kc * 8;
      sok = c < A.C && zok;
      sbase = !sok ? s0 : (c < d.C0) ? s0 + c : s1 + (c - d.C0);
      scs = (c < d.C0) ? d.C0 : d.C1;
      simg = sl * HWs + poff;
      sca = sok ? c : ZCOEF;
      scb = sok ? A.C + c : ZCOEF;
    } else {
      const int c = (chunk - A.nchunk1) * BK + kc * 8;
      sok = c < A.C23;
      sbase = !sok ? s2 : (c < d.C2) ? s2 + c : s3 + (c - d.C2);
      scs = (c < d.C2) ? d.C2 : d.C3;
      simg = 0;
      sca = ZCOEF;
      scb = ZCOEF;
    }
  };
  u32x4 rh[SL];
  int roff[SL];
  // staging round q of a 3x3 chunk (1x1 chunks: stage_seg2)
  auto load_round = [&](int q) {
    const int sp = spix[q];
    const bool valid = sok && sp >= 0;
    const bf16r* src = valid ? sbase + (size_t)(simg + sp) * scs : s0;
    rh[q % SL] = HDBG9(1) ? u32x4{0u, 0u, 0u, 0u} : *(const u32x4*)src;
    // GN prologue: padding positions were zeroed once (their store goes to the dummy slot) and invalid channels /
    // depth slices meet zero coefficients, so the transform needs no select
    const int dst = sdst0 + q * 1024;
    roff[q % SL] = sp == -2 ? DUMMY : PRO != 0 ? (sp >= 0 ? dst : DUMMY) : (dst | (valid ? 0 : ZFLAG));
  };
  auto transform = [&](int q) -> u32x4 {
    const u32x4 raw = rh[q % SL];
    u32x4 v = raw;
    if (PRO != 0 && !HDBG9(2)) {
      const f32x4 a0 = *(const f32x4*)(coef + sca), a1 = *(const f32x4*)(coef + sca + 4);
      const f32x4 b0 = *(const f32x4*)(coef + scb), b1 = *(const f32x4*)(coef + scb + 4);
      const float qa[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const float qb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#if FMD_H9_FENCE
      // the 8 elements advance stage by stage (register fences), not element by element
      float y[8], t[8];
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        y[2 * e] = bf_lo(raw[e]) * qa[2 * e] + qb[2 * e];
        y[2 * e + 1] = bf_hi(raw[e]) * qa[2 * e + 1] + qb[2 * e + 1];
      }
      if (PRO == 2) {
        fence8_(y);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_exp2f(y[i] * -1.4426950408889634f);
        fence8_(t);
#pragma unroll
        for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_rcpf(1.f + t[i]);
        fence8_(t);
#pragma unroll
        for (int i = 0; i < 8; ++i) y[i] = y[i] * t[i];
      }
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = pack2(y[2 * e], y[2 * e + 1]);
#else
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = bf_lo(raw[e]) * qa[2 * e] + qb[2 * e];
        float hi = bf_hi(raw[e]) * qa[2 * e + 1] + qb[2 * e + 1];
        if (PRO == 2) { lo = siluf_(lo); hi = siluf_(hi); }
        v[e] = pack2(lo, hi);
      }
#endif
    } else {
      const bool z = (roff[q % SL] & ZFLAG) != 0;
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = z ? 0u : v[e];
    }
    return v;
  };

  // ---- A fragments: 8 pixel blocks of the wave (rows 2pb, 2pb+1), one k-step of a tap
  int abase;
  int uo[9];
  if constexpr (UP) {
    abase = (hh * HPAD + HROW + 1) * 16;
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      const int ky = t / 3, kx = t % 3;
      uo[t] = (((rr + ky - 1) >> 1) * HROW + ((col + kx - 1) >> 1)) * 16;
    }
  } else {
    abase = (hh * HPAD + rr * HROW + col) * 16;
#pragma unroll
    for (int t = 0; t < 9; ++t) uo[t] = 0;
  }
  auto aoff = [&](int tap, int s, int pb) {
    const int ky = MODE ? tap >> 1 : tap / 3, kx = MODE ? tap & 1 : tap % 3;
    return UP ? abase + uo[tap] + (s * 2 * HPAD + pb * HROW) * 16
              : abase + (s * 2 * HPAD + (2 * pb + ky) * HROW + kx) * 16;
  };

  f32x16 acc[NPB];
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
    for (int e = 0; e < 16; ++e) acc[pb][e] = 0.f;

  // one tap: 8 pixel blocks x 2 k-steps = 16 MFMAs.  The 16 A-fragment reads are software-pipelined four
  // groups ahead of their MFMAs (sched_group_barrier: 8 reads, then 4 MFMAs + 4 reads per group), so each group's
  // LDS latency hides under the previous group's 4 x 32 MFMA cycles instead of every MFMA waiting on its read
  auto tap_mma = [&](int tap, int hb, const bf16x8 (&bq)[2]) {
    bf16x8 af[2 * NPB];
    if constexpr (NPB < 4) {   // 4-row tiles: both k-halves' reads, then their MFMAs
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) af[s * NPB + pb] = *(const bf16x8*)(smem + hb + aoff(tap, s, pb));
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) acc[pb] = mfma32(af[s * NPB + pb], bq[s], acc[pb]);
      return;
    }
    constexpr int NG = NPB / 4 > 0 ? NPB / 4 : 1;   // groups of 4 pixel blocks per k-half
#pragma unroll
    for (int g = 0; g < 2 * NG; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) af[4 * g + i] = *(const bf16x8*)(smem + hb + aoff(tap, g / NG, 4 * (g % NG) + i));
#pragma unroll
    for (int g = 0; g < 2 * NG; ++g)
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[4 * (g % NG) + i] = mfma32(af[4 * g + i], bq[g / NG], acc[4 * (g % NG) + i]);
    if constexpr (H9_SCHED && NPB == 8) {
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    }
  };
  auto next_chunk = [&](int c) { return c + 1 < c_hi ? c + 1 : (c + 1 == c_hi && n_seg2 ? A.nchunk1 : -1); };
  // a 1x1 chunk (raw src2 | src3 at the tile's own pixels) staged whole into buffer byte offset buf
  auto stage_seg2 = [&](int ch, int buf) {
    setup(ch);
    u32x4 sv[4];
#pragma unroll
    for (int q = 0; q < THT / 4; ++q) sv[q] = *(const u32x4*)(sok ? sbase + (size_t)(s2pix0 + 4 * q * d.Wo) * scs : s2);
#pragma unroll
    for (int q = 0; q < THT / 4; ++q)
      *(u32x4*)(smem + buf + s2dst0 + q * 72 * 16) = sok ? sv[q] : u32x4{0u, 0u, 0u, 0u};
  };

  // ---- prologue: padding positions of both halo buffers zeroed (fixed for the tile); first chunk staged whole;
  // B of its tap 0 in flight
#pragma unroll
  for (int q = 0; q < NR; ++q)
    if (spix[q] == -1) {
      *(u32x4*)(smem + sdst0 + q * 1024) = u32x4{0u, 0u, 0u, 0u};
      *(u32x4*)(smem + HBUF + sdst0 + q * 1024) = u32x4{0u, 0u, 0u, 0u};
    }
  __syncthreads();   // affine + epilogue tables
  if (A.splits <= 1) {   // the summed bias is the accumulators' start value
    const float bv = epi[32 * wid + r];
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[pb][e] = bv;
  }
  // B fragments three slots deep: the load of slot g + 2 is issued at slot g, two taps (about 2,000 cycles with
  // the partner wave) ahead of its MFMAs -- one tap did not cover an L2 hit under load
  bf16x8 bq[RB][2];
  const int last2 = T1 + n_seg2 - 1;   // last 1x1 slot of this split (when n_seg2 > 0)
  if (c_lo < c_hi) {
    loadB(bq[0], c_lo * NTAP);
    loadB(bq[1], c_lo * NTAP + 1);
  } else {
    loadB(bq[0], T1);
    loadB(bq[1], min(T1 + 1, last2));
  }
  if (c_lo >= c_hi) {
    if (n_seg2) stage_seg2(A.nchunk1, (A.nchunk1 & 1) * HBUF);
  } else {
    setup(c_lo);
    u32x4 pv[NR];
    int po[NR];
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      load_round(q);
      pv[q] = rh[q % SL];
      po[q] = roff[q % SL];
    }
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      rh[q % SL] = pv[q];
      roff[q % SL] = po[q];
      const u32x4 v = transform(q);
      *(u32x4*)(smem + (c_lo & 1) * HBUF + (roff[q % SL] & ~ZFLAG)) = v;
    }
  }
  __syncthreads();

  for (int chunk = c_lo; chunk < c_hi; ++chunk) {
    const int nx = next_chunk(chunk);
    const int hb = (chunk & 1) * HBUF, nb = ((chunk + 1) & 1) * HBUF;
    // next chunk a 3x3 one: staged in rounds under this chunk's taps (the 1x1 segment's first chunk is staged
    // whole after the loop); B of the next chunk's tap 0 / the first 1x1 slot at the last tap
    const bool stg = nx >= 0 && nx < A.nchunk1;
    if (stg) setup(nx);
    // S2D: this chunk's plane (a, b) reads halo rows / columns {0, +1} where a / b = 0; D2S: always {0, +1}
    int hadj = D2S ? HROW * 16 + 16 : 0;
    if (S2D) {
      const int pl = (chunk % (4 * A.ncb)) / A.ncb;
      hadj = ((pl >> 1) ? 0 : HROW * 16) + ((pl & 1) ? 0 : 16);
    }
#pragma unroll
    for (int t = 0; t < NTAP; ++t) {
      // slot of tap t + 2: this chunk, the next 3x3 chunk's taps 0 / 1, the first 1x1 slots, or a re-load
      const int s2 = t < NTAP - 2 ? chunk * NTAP + t + 2
                     : stg ? nx * NTAP + t - (NTAP - 2) : nx < 0 ? chunk * NTAP + t : min(T1 + t - (NTAP - 2), last2);
      if (!HDBG9(8)) loadB(bq[(t + 2) % RB], s2);
      if (stg) {
        // rounds loaded LAG taps ago leave their register slots before this tap's rounds land in them
#pragma unroll
        for (int j = 0; j < RPT; ++j) {
          const int q = (t - LAG) * RPT + j;
          if (t >= LAG && q < NR) {
            const u32x4 v = transform(q);
            *(u32x4*)(smem + nb + (roff[q % SL] & ~ZFLAG)) = v;
          }
        }
#pragma unroll
        for (int j = 0; j < RPT; ++j)
          if (t * RPT + j < NR) load_round(t * RPT + j);
      }
      if (!HDBG9(256)) tap_mma(t, hb + hadj, bq[t % RB]);
    }
    // chunk boundary: the next chunk's halo complete, this chunk's buffer free (NTAP % RB == 0: the B ring's phase
    // is the same at every chunk start)
    __syncthreads();
  }
  if (c_lo < c_hi && n_seg2) {   // first 1x1 chunk, staged whole after the 3x3 chunks (its buffer is free)
    stage_seg2(A.nchunk1, (A.nchunk1 & 1) * HBUF);
    __syncthreads();
  }

  // ---- 1x1 chunks: one tap each; the next chunk loaded whole; B of the next slot one step ahead
  for (int i = 0; i < n_seg2; ++i) {
    const int ch = A.nchunk1 + i;
    const bool more = i + 1 < n_seg2;
    setup(more ? ch + 1 : -1);
    loadB(bq[2], min(T1 + i + 2, last2));
    u32x4 sv[THT / 4];
    int so[THT / 4];
#pragma unroll
    for (int q = 0; q < THT / 4; ++q) {
      const bool valid = more && sok;
      const bf16r* src = valid ? sbase + (size_t)(s2pix0 + 4 * q * d.Wo) * scs : s2;
      sv[q] = *(const u32x4*)src;
      so[q] = !more ? DUMMY : (s2dst0 + q * 72 * 16) | (valid ? 0 : ZFLAG);
    }
    tap_mma(4, (ch & 1) * HBUF, bq[0]);
#pragma unroll
    for (int q = 0; q < THT / 4; ++q) {
      u32x4 v = sv[q];
      if (so[q] & ZFLAG) v = u32x4{0u, 0u, 0u, 0u};
      *(u32x4*)(smem + ((ch + 1) & 1) * HBUF + (so[q] & ~ZFLAG)) = v;
    }
    __syncthreads();
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      bq[0][h] = bq[1][h];
      bq[1][h] = bq[2][h];
    }
  }

  if (HDBG9(4)) return;
  // ------------------------------------------------------------ epilogue (layout of v9; wave = cout quarter)
  const int K = d.K, Ho = d.Ho, Wo = d.Wo;
  auto pixl = [&](int pb, int pr) {
    const int q = pr >> 4;
    const int cl = q ? ((pr - 18) & 15) : pr;
    return (2 * pb + q) * TW + cl;
  };
  if constexpr (THT <= 8 && MODE == 0) {   // (compiled only where its registers fit: the 8- and 4-row 3x3 tiles)
  if (A.splits > 1 && d.tickets) {
    // Split-K combined inside the launch (MI355X_MICROARCH.md, inter-workgroup visibility: a counter hand-off with a
    // write-through payload; the same protocol as csrc/conv_small.hip).  Each part stores its accumulators in their
    // register layout (16-byte pieces [part][pixel block][quarter][thread] of the tile's slab of d.ws) with sc1
    // stores, every wave drains them, then ONE lane takes the tile's ticket; the part drawing splits - 1 resets it
    // and sums the parts in part order (its own from registers, the same values it stored), so the result does not
    // depend on which part arrives last, then runs the unsplit epilogue below.
    constexpr int SLOT = NPB * 16;   // floats per thread and part
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(d.ws + (size_t)b * A.splits * NT9 * SLOT, 0,
                                                      A.splits * NT9 * SLOT * 4, 0x00020000);
    auto piece = [&](int s, int pb, int j) { return (((s * NPB + pb) * 4 + j) * NT9 + tid) * 16; };
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const f32x4 v = f32x4{acc[pb][4 * j], acc[pb][4 * j + 1], acc[pb][4 * j + 2], acc[pb][4 * j + 3]};
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v), rs, piece(split, pb, j), 0, 16);
      }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* const last = (int*)coef;   // the affine table is dead after the chunk loop; the epilogue does not touch it
    if (tid == 0) {
      auto* tk = (__attribute__((address_space(1))) unsigned*)(d.tickets + b);
      const unsigned t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = t == (unsigned)(A.splits - 1);
      if (is_last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = is_last;
    }
    __syncthreads();
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f32x16 tot[NPB];
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int e = 0; e < 16; ++e) tot[pb][e] = 0.f;
    for (int s = 0; s < A.splits; ++s) {
      if (s == split) {
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb) tot[pb] += acc[pb];
      } else {
        u32x4 v[NPB * 4];
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
          for (int j = 0; j < 4; ++j) v[pb * 4 + j] = __builtin_amdgcn_raw_buffer_load_b128(rs, piece(s, pb, j), 0, 16);
#pragma unroll
        for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const f32x4 f = __builtin_bit_cast(f32x4, v[pb * 4 + j]);
#pragma unroll
            for (int e = 0; e < 4; ++e) tot[pb][4 * j + e] += f[e];
          }
      }
    }
    const float bv = epi[32 * wid + r];   // the summed bias, after the parts
#pragma unroll
    for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
      for (int e = 0; e < 16; ++e) acc[pb][e] = tot[pb][e] + bv;
  }
  }
  if (A.splits > 1 && !(THT <= 8 && MODE == 0 && d.tickets)) {
    float* ws = d.ws + (size_t)split * d.N * Ho * Wo * K;
    const int co = co0 + 32 * wid + r;
    if (co < K) {
#pragma unroll
      for (int pb = 0; pb < NPB; ++pb)
#pragma unroll
        for (int e = 0; e < 16; ++e) {
          const int pi = pixl(pb, (e & 3) + 8 * (e >> 2) + 4 * hh);
          ws[(size_t)opix(pi) * K + co] = acc[pb][e];
        }
    }
    return;
  }
  unsigned char* const tileb = smem;
  const bool hasx = d.ep_x0 != nullptr;
  const bool dep = d.ep_a != nullptr;
  const bool side = d.resid != nullptr || hasx;
  const bool stats = d.stats != nullptr;
  // side input (residual / the data gradient's x) of pixel block pb = tile rows 2pb, 2pb+1: two 16-byte pieces per
  // thread, loaded two pixel blocks ahead of their use and staged into the block's rows of the output tile
  auto side_piece = [&](int k) -> const bf16r* {
    const int q = tid + NT9 * k, pi = q >> 4, c16 = q & 15;
    const int p = opix(pi);
    const int c = co0 + c16 * 8;
    return d.resid ? (const bf16r*)d.resid + (size_t)p * K + c
                   : (c < d.ep_C0) ? (const bf16r*)d.ep_x0 + (size_t)p * d.ep_C0 + c
                                   : (const bf16r*)d.ep_x1 + (size_t)p * (K - d.ep_C0) + (c - d.ep_C0);
  };
  u32x4 sv[2][2];
  if (side) {
#pragma unroll
    for (int k = 0; k < 4; ++k) sv[k >> 1][k & 1] = *(const u32x4*)side_piece(k);
  }
  bf16x8 inat[2], iperm[2];
#pragma unroll
  for (int s = 0; s < 2; ++s)
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      inat[s][j] = (__bf16)((16 * s + 8 * hh + j) == r ? 1.0f : 0.0f);
      iperm[s][j] = (__bf16)((16 * s + 8 * (j >> 2) + 4 * hh + (j & 3)) == r ? 1.0f : 0.0f);
    }
  const int cl = 32 * wid;
  const float ea = epi[BCO + cl + r], eb = epi[2 * BCO + cl + r];
  float st1 = 0.f, st2 = 0.f;
#pragma unroll
  for (int pb = 0; pb < NPB; ++pb) {
    const int pi_l = pixl(pb, r);
    f32x16 v = acc[pb];
    f32x16 xc;
    if (side) {
#pragma unroll
      for (int j = 0; j < 2; ++j) {
        const int q = tid + NT9 * (2 * pb + j), pi = q >> 4, c16 = q & 15;
        *(u32x4*)(tileb + pi * 256 + ((c16 ^ (pi & 15)) * 16)) = sv[pb & 1][j];
      }
      __syncthreads();
      if (pb + 2 < NPB) {
#pragma unroll
        for (int j = 0; j < 2; ++j) sv[pb & 1][j] = *(const u32x4*)side_piece(2 * pb + 4 + j);
      }
      bf16x8 fr[2];
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const int c = cl + 16 * s + 8 * hh;
        fr[s] = *(const bf16x8*)(tileb + pi_l * 256 + (((c >> 3) ^ (pi_l & 15)) * 16));
      }
      if (d.resid) {
#pragma unroll
        for (int s = 0; s < 2; ++s) v = mfma32(fr[s], inat[s], v);
      } else {
#pragma unroll
        for (int e = 0; e < 16; ++e) xc[e] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) xc = mfma32(fr[s], inat[s], xc);
      }
    }
    if (hasx && dep) {
#pragma unroll
      for (int e = 0; e < 16; ++e) v[e] *= silu_grad(ea * xc[e] + eb);
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
          st2 += hasx ? w0 * xc[8 * s + 2 * e] + w1 * xc[8 * s + 2 * e + 1] : w0 * w0 + w1 * w1;
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
    if (stats && (pb & 1)) {   // one statistics row per 64 pixels (= pixel blocks 2k, 2k+1: 4 tile rows)
      const int srow = (D2S ? tile * (A.depth ? 8 : 4) + ocls : tile) * (THT * TW / 64) + (pb >> 1);
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
  for (int k = 0; k < THT * TW * BCO / 8 / NT9; ++k) {
    const int q = tid + NT9 * k, pi = q >> 4, c16 = q & 15;
    *(u32x4*)((bf16r*)d.out + (size_t)opix(pi) * K + co0 + c16 * 8) =
        *(const u32x4*)(tileb + pi * 256 + ((c16 ^ (pi & 15)) * 16));
  }
}

}  // namespace

namespace {
// grids of fewer workgroups than this (16-row tiles x splits) run 8-row tiles: at 128^2 / 64^2 a 16-row grid is one
// round of 512 (or 256) workgroups whose prologues and epilogues all coincide (0 = never)
int g_th8_max_wg = 1024;
// 8-row grids (tiles x splits) of fewer workgroups than this run 4-row tiles (plain 3x3 only; 0 = never): the latent
// UNet's 32^2 convs are 64 tiles x 2-4 parts on 256 CUs (config D 121.6 -> 124.8 (256) -> 126.5 img/s (512); 1024 takes
// the config B sampler's 64^2 level too: 26.2 -> 25.5 img/s)
int g_th4_max_wg = 512;

template <int THT>
int halo9_go(const HArgs& A, int pro, fmd_stream_t stream) {
  const int nwg = A.d.N * A.tiles_x * A.tiles_y * A.ntc;
  const dim3 g(nwg, A.splits);
  const dim3 blk(NT9);
  hipStream_t st = (hipStream_t)stream;
  if (A.d.upsample) {
    if (pro == 2) hipLaunchKernelGGL((conv3x3_halo9b<true, 2, 0, THT>), g, blk, 0, st, A);
    else if (pro == 1) hipLaunchKernelGGL((conv3x3_halo9b<true, 1, 0, THT>), g, blk, 0, st, A);
    else hipLaunchKernelGGL((conv3x3_halo9b<true, 0, 0, THT>), g, blk, 0, st, A);
  } else {
    if (pro == 2) hipLaunchKernelGGL((conv3x3_halo9b<false, 2, 0, THT>), g, blk, 0, st, A);
    else if (pro == 1) hipLaunchKernelGGL((conv3x3_halo9b<false, 1, 0, THT>), g, blk, 0, st, A);
    else hipLaunchKernelGGL((conv3x3_halo9b<false, 0, 0, THT>), g, blk, 0, st, A);
  }
  return (int)hipGetLastError();
}
}  // namespace

extern "C" int fmd_halo_set_th8_max_workgroups(int32_t n) {
  g_th8_max_wg = n < 0 ? 0 : n;
  return 0;
}

int halo9_launch(const HArgs& A, int pro, fmd_stream_t stream) {
  const fmd_conv_desc* d = &A.d;
  if (d->gout) return 1;
  if (d->upsample && d->src2) return 1;
  const bool tk = A.splits > 1 && d->tickets;   // split-K with the in-launch combine and the unsplit epilogue
  if ((A.splits <= 1 || tk) && (d->K % BCO || d->out_f32 || d->accumulate || (d->resid && d->ep_x0))) return 1;
  if (A.splits > 1 && (d->out_f32 || d->accumulate)) return 1;
  if (tk && (A.depth || d->n_tickets < (long long)A.d.N * A.tiles_x * (d->Ho / 4) * A.ntc ||
             (d->stats && d->tickets_rows != 64)))
    return 1;
  const long long nwg16 = (long long)A.d.N * A.tiles_x * A.tiles_y * A.ntc * A.splits;
  if (tk && !(nwg16 < g_th8_max_wg && d->Ho % 8 == 0)) return 1;   // the combine exists in the 8- and 4-row instances
  if (nwg16 < g_th8_max_wg && d->Ho % 8 == 0) {
    HArgs A8 = A;
    A8.tiles_y = d->Ho / 8;
    if (2 * nwg16 < g_th4_max_wg && !A.depth) {   // 4-row tiles: twice the 8-row grid, still under one round
      A8.tiles_y = d->Ho / 4;
      return halo9_go<4>(A8, pro, stream);
    }
    return halo9_go<8>(A8, pro, stream);
  }
  return halo9_go<TH>(A, pro, stream);
}

extern "C" int fmd_halo_set_th4_max_workgroups(int32_t n) {
  g_th4_max_wg = n < 0 ? 0 : n;
  return 0;
}

// ---------------------------------------------------------------------------------------------------------------
// Stride-2 pad-1 convs on the space-to-depth halo kernel (conv3x3_halo9b<false, PRO, true>).

namespace {

// tap index u of the ks-tap stride-2 kernel that plane parity a meets at its i-th halo offset (i = 0, 1):
// a = 0 -> offsets {0, +1} = taps 1, 3; a = 1 -> offsets {-1, 0} = taps 0, 2
FMD_DEV int s2d_tap(int a, int i) { return a ? 2 * i : 1 + 2 * i; }

// out[tco][chunk][tap][kc][co 128][8] bf16 (the halo tiling of a 2x2 conv)
//   mode 0 (forward, ks = 3 or 4): rows = K couts, inner = 4C plane-major; value w[co][c][u][v] (0 where u or v >= ks)
//   mode 1 (data gradient of conv3x3(nearest_x2(x))): rows = C, inner = 4K; the 4x4 kernel the nearest-x2 copy
//            folds the 3x3 into, W4[c][k][u][v] = sum_{ky in S(u), kx in S(v)} w[k][c][ky][kx],
//            S(0) = {2}, S(1) = {1, 2}, S(2) = {0, 1}, S(3) = {0}
//   mode 2 (data gradient of a stride-2 3x3, D2S): rows = 4C class-major, inner = K; class a meets dy offset u with
//            tap ky = (a ? (u ? 0 : 2) : (u ? none : 1)), columns alike
// 3-D masters (d3, [K][C][3][3][3]): the chunks gain a leading depth index -- mode 0 the depth tap kz < 3, mode 1 the
// folded depth tap kz < 4 (S(kz) as in-plane), mode 2 the depth offset dz < 2 with 8 classes (depth parity c = class
// >> 2 meeting dz with tap kd = c ? (dz ? 0 : 2) : (dz ? none : 1))
__host__ __device__ inline int s2d_depth_groups(int mode, int ks, int d3) { return !d3 ? 1 : mode == 0 ? ks : mode == 1 ? 4 : 2; }

__global__ void s2d_tile_weights_kernel(const float* __restrict__ w, int K, int C, int ks, int mode, int d3,
                                        bf16r* __restrict__ out, long long total) {
  const long long e = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= total) return;
  const int R = mode == 0 ? K : mode == 1 ? C : (d3 ? 8 : 4) * C, Ci = mode == 0 ? C : K;
  const int nch2 = (mode == 2 ? Ci : 4 * Ci) / BK;   // chunks per depth group
  const int nch = s2d_depth_groups(mode, ks, d3) * nch2;
  const int kt = d3 ? 3 : 1;                          // depth extent of the master
  long long t = e;
  const int j = (int)(t % 8); t /= 8;
  const int co = (int)(t % BCO); t /= BCO;
  const int kc = (int)(t % KC); t /= KC;
  const int tap = (int)(t % 4); t /= 4;
  const int chunk = (int)(t % nch); t /= nch;
  const int tco = (int)t;
  const int row = tco * BCO + co;
  const int kz = chunk / nch2;
  const int ch = (chunk - kz * nch2) * BK + kc * 8 + j;   // inner channel (modes 0, 1: plane-major over 4*Ci)
  float val = 0.f;
  if (mode == 2) {
    const int cls = row / C, c = row - cls * C;
    const int a = (cls >> 1) & 1, b = cls & 1, uu = tap >> 1, vv = tap & 1;
    const int ky = a ? (uu ? 0 : 2) : (uu ? -1 : 1), kx = b ? (vv ? 0 : 2) : (vv ? -1 : 1);
    const int kd = !d3 ? 0 : (cls >> 2) ? (kz ? 0 : 2) : (kz ? -1 : 1);
    if (row < R && ky >= 0 && kx >= 0 && kd >= 0) val = w[((((size_t)ch * C + c) * kt + kd) * 3 + ky) * 3 + kx];
    out[e] = (bf16r)f2bf(val);
    return;
  }
  const int pl = ch / Ci, ci = ch - pl * Ci;
  const int u = s2d_tap(pl >> 1, tap >> 1), v = s2d_tap(pl & 1, tap & 1);
  if (row < R) {
    if (!mode) {
      if (u < ks && v < ks) val = w[((((size_t)row * C + ci) * kt + kz) * ks + u) * ks + v];
    } else {
      auto lo = [](int q) { return q == 0 ? 2 : q == 3 ? 0 : 2 - q; };
      auto hi = [](int q) { return q == 0 ? 2 : q == 3 ? 0 : 3 - q; };
      const int dlo = d3 ? lo(kz) : 0, dhi = d3 ? hi(kz) : 0;
      for (int kd = dlo; kd <= dhi; ++kd)
        for (int ky = lo(u); ky <= hi(u); ++ky)
          for (int kx = lo(v); kx <= hi(v); ++kx) val += w[((((size_t)ci * C + row) * kt + kd) * 3 + ky) * 3 + kx];
    }
  }
  out[e] = (bf16r)f2bf(val);
}

}  // namespace

extern "C" int64_t fmd_s2d_tiled_size_nd(int32_t K, int32_t C, int32_t mode, int32_t ks, int32_t dims) {
  const int d3 = dims == 3;
  const int64_t R = mode == 0 ? K : mode == 1 ? C : (d3 ? 8LL : 4LL) * C, Ci = mode == 0 ? C : K;
  return ((R + BCO - 1) / BCO) * s2d_depth_groups(mode, ks, d3) * ((mode == 2 ? Ci : 4 * Ci) / BK) * 4 * KC * BCO * 8;
}

extern "C" int64_t fmd_s2d_tiled_size(int32_t K, int32_t C, int32_t mode) {
  return fmd_s2d_tiled_size_nd(K, C, mode, 3, 2);
}

extern "C" int fmd_s2d_tile_weights_nd(const float* w, int32_t K, int32_t C, int32_t ks, int32_t mode, int32_t dims,
                                       void* out, fmd_stream_t stream) {
  const int Ci = mode ? K : C;
  if (dims != 2 && dims != 3) return -1;
  if (mode < 0 || mode > 2 || (mode == 0 && ks != 3 && ks != 4) || (mode != 0 && ks != 3) || Ci % BK) return -1;
  if (dims == 3 && ks != 3) return -1;
  if (mode == 2 && C % BCO) return -1;   // one output class per 128-row tile
  const long long total = fmd_s2d_tiled_size_nd(K, C, mode, ks, dims);
  hipLaunchKernelGGL(s2d_tile_weights_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0,
                     (hipStream_t)stream, w, K, C, ks, mode, (int)(dims == 3), (bf16r*)out, total);
  return (int)hipGetLastError();
}

extern "C" int fmd_s2d_tile_weights(const float* w, int32_t K, int32_t C, int32_t ks, int32_t mode, void* out,
                                    fmd_stream_t stream) {
  return fmd_s2d_tile_weights_nd(w, K, C, ks, mode, 2, out, stream);
}

extern "C" int fmd_conv_s2d(const fmd_conv_desc* d, fmd_stream_t stream) {
  if (d->stride != 2 || d->pad != 1 || (d->ks != 3 && d->ks != 4) || d->transposed || d->upsample) return 1;
  const bool d3 = d->Do > 0 || d->Ds > 0;   // 3-D: the depth taps as chunks (kz, plane, block)
  if (d3 && d->Ds != 2 * d->Do) return 1;
  if (d->src2 || d->gout || d->out_f32 || d->splits > 1 || d->fold_st0) return 1;
  if (d->Hs != 2 * d->Ho || d->Ws != 2 * d->Wo || d->Ho % TH || d->Wo % TW) return 1;
  const int C = d->C0 + d->C1;
  if (C % BK || d->C0 % 8 || d->K % BCO || !d->wgt_tiled) return 1;
  if (d->pro_a && C > CMAX) return 1;
  if (d->accumulate && (d->resid || d->ep_x0)) return 1;
  const long long Ns = (long long)d->N * (d3 ? d->Ds : 1), No = (long long)d->N * (d3 ? d->Do : 1);
  if (Ns * d->Hs * d->Ws * (d->C0 > d->C1 ? d->C0 : d->C1) >= (1LL << 31) ||
      No * d->Ho * d->Wo * d->K >= (1LL << 31)) return 1;
  HArgs A;
  A.d = *d;
  if (d->accumulate) {   // out += conv: the old output enters as the residual side input of the same tile
    A.d.resid = d->out;
    A.d.accumulate = 0;
  }
  A.d.N = (int)No;           // images: the output (depth) slices
  A.C = C;
  A.C23 = 0;
  A.tiles_x = d->Wo / TW;
  A.tiles_y = d->Ho / TH;
  A.ntc = d->K / BCO;
  A.depth = d3 ? d->Do : 0;
  A.dsrc = d3 ? d->Ds : 0;
  A.ncb = C / BK;                              // chunks per plane
  A.nchunk1 = (d3 ? d->ks : 1) * 4 * A.ncb;    // (depth tap,) plane-major
  A.nchunk2 = 0;
  A.nsteps_slots = A.nchunk1 * 4;
  A.splits = 1;
  A.cps = A.nchunk1;
  A.wt = (const bf16r*)d->wgt_tiled;
  A.wt2 = nullptr;
  A.tbuf = nullptr;
  A.dbg = 0;
  const int nwg = A.d.N * A.tiles_x * A.tiles_y * A.ntc;
  if (nwg < 128) return 1;
  const int pro = d->pro_a ? (d->pro_silu ? 2 : 1) : 0;
  hipStream_t st = (hipStream_t)stream;
  if (nwg < g_th8_max_wg) {   // 8-row tiles on a one-round grid (as halo9_launch)
    A.tiles_y = d->Ho / 8;
    const dim3 g(2 * nwg), blk(NT9);
    if (pro == 2) hipLaunchKernelGGL((conv3x3_halo9b<false, 2, 1, 8>), g, blk, 0, st, A);
    else if (pro == 1) hipLaunchKernelGGL((conv3x3_halo9b<false, 1, 1, 8>), g, blk, 0, st, A);
    else hipLaunchKernelGGL((conv3x3_halo9b<false, 0, 1, 8>), g, blk, 0, st, A);
    return (int)hipGetLastError();
  }
  const dim3 g(nwg), blk(NT9);
  if (pro == 2) hipLaunchKernelGGL((conv3x3_halo9b<false, 2, 1>), g, blk, 0, st, A);
  else if (pro == 1) hipLaunchKernelGGL((conv3x3_halo9b<false, 1, 1>), g, blk, 0, st, A);
  else hipLaunchKernelGGL((conv3x3_halo9b<false, 0, 1>), g, blk, 0, st, A);
  return (int)hipGetLastError();
}

extern "C" int fmd_conv_d2s(const fmd_conv_desc* d, fmd_stream_t stream) {
  if (!d->transposed || d->stride != 2 || d->pad != 1 || d->ks != 3 || d->upsample) return 1;
  const bool d3 = d->Do > 0 || d->Ds > 0;   // 3-D: 8 output classes, chunks (depth offset, block)
  if (d3 && d->Do != 2 * d->Ds) return 1;
  if (d->src2 || d->gout || d->out_f32 || d->splits > 1 || d->pro_a || d->fold_st0) return 1;
  if (d->Ho != 2 * d->Hs || d->Wo != 2 * d->Ws || d->Hs % TH || d->Ws % TW) return 1;
  const int C = d->C0 + d->C1;
  if (C % BK || d->C0 % 8 || d->K % BCO || !d->wgt_tiled) return 1;
  if (d->accumulate && (d->resid || d->ep_x0)) return 1;
  const long long Ns = (long long)d->N * (d3 ? d->Ds : 1), No = (long long)d->N * (d3 ? d->Do : 1);
  if (Ns * d->Hs * d->Ws * (d->C0 > d->C1 ? d->C0 : d->C1) >= (1LL << 31) ||
      No * d->Ho * d->Wo * d->K >= (1LL << 31)) return 1;
  HArgs A;
  A.d = *d;
  if (d->accumulate) {
    A.d.resid = d->out;
    A.d.accumulate = 0;
  }
  A.d.N = (int)Ns;           // images: the gradient's (depth) slices
  A.C = C;
  A.C23 = 0;
  A.tiles_x = d->Ws / TW;    // tiles over the low-resolution input grid; 4 (3-D: 8) output classes per tile
  A.tiles_y = d->Hs / TH;
  A.ntc = (d3 ? 8 : 4) * (d->K / BCO);
  A.depth = d3 ? d->Ds : 0;
  A.dsrc = d3 ? d->Ds : 0;
  A.ncb = C / BK;
  A.nchunk1 = (d3 ? 2 : 1) * A.ncb;
  A.nchunk2 = 0;
  A.nsteps_slots = A.nchunk1 * 4;
  A.splits = 1;
  A.cps = A.nchunk1;
  A.wt = (const bf16r*)d->wgt_tiled;
  A.wt2 = nullptr;
  A.tbuf = nullptr;
  A.dbg = 0;
  const int nwg = A.d.N * A.tiles_x * A.tiles_y * A.ntc;
  if (nwg < 128) return 1;
  if (nwg < g_th8_max_wg) {   // 8-row tiles on a one-round grid (as halo9_launch)
    A.tiles_y = d->Hs / 8;
    hipLaunchKernelGGL((conv3x3_halo9b<false, 0, 2, 8>), dim3(2 * nwg), dim3(NT9), 0, (hipStream_t)stream, A);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL((conv3x3_halo9b<false, 0, 2>), dim3(nwg), dim3(NT9), 0, (hipStream_t)stream, A);
  return (int)hipGetLastError();
}
