// Small-level convolution in one launch (fmd_conv_small): the sampler's low-resolution UNet levels.
//
// Why: at 16^2 ... 1^2 a conv moves a few MB and its MFMA work is a few microseconds of one CU,
// so the split-K implicit GEMM of csrc/conv.hip spent its time at the ~5 us launch floor three or four times per conv
// (main launch, split-K combine, GroupNorm statistics / affine, materialised GN+SiLU operand).  Here one launch does
// it all:
//
// * tile = up to 64 output pixels (a 64-pixel block of one image: 64 / Wo rows, or S whole images when Ho*Wo < 64)
//   x 16 or 32 output channels; 512 threads = 8 waves, one workgroup per CU (LDS up to 160 KiB).  Where that leaves
//   fewer than 256 workgroups the reduction (input channels, whole GroupNorm groups) is split into P parts, one
//   workgroup each, combined inside the launch (below);
// * prologue: every global operand is in flight at once -- the wave's weight fragments (buffer loads straight into
//   registers, branch-free), and by LDS-DMA the input rows the tile's taps read (the part's channels of the virtual
//   concat C0 | C1, [pixel slot][channel] rows with a 16-byte-chunk XOR swizzle), the raw 1x1-segment input, the
//   producers' GroupNorm statistics slab rows, gamma / beta / scale-shift rows and the epilogue operands;
// * GroupNorm: the affine of every input channel folded from the statistics (E[x^2] - mean^2, group sums in fp64 by
//   a butterfly over the group's lanes), the scale-shift embedding folded in; applied + SiLU in place in LDS;
// * main loop: waves split the 32-channel chunks (and the 16-pixel row blocks); per chunk 9 taps (1 for mode 3) x
//   row blocks of v_mfma_f32_16x16x32_bf16, A = weights (registers), B = the staged pixels (ds_read_b128);
// * epilogue: the waves' partial tiles meet in LDS in a fixed order (deterministic); with P > 1 every part stores its
//   fp32 tile write-through (sc1) and takes a ticket, the last part sums all P in part order (the result does not
//   depend on arrival order); + bias / skip bias / per-sample bias / residual, bf16 16-byte stores, and the
//   per-channel statistics of the rounded outputs (the slab rows the consumer's GroupNorm folds).
//
// Measured: each workgroup's phases are latency chains of a few microseconds each, so a launch
// costs ~15 us whatever its size; it replaces three to four launches at the ~5 us floor.
#include <cstdlib>
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

#ifndef FMD_SMALL_NT
#define FMD_SMALL_NT 512
#endif
// 8 waves per workgroup, one workgroup per CU.  -DFMD_SMALL_NT=256 builds 4-wave workgroups, two per CU where the
// LDS plan allows, whose phases run out of step: measured no better on the latent UNet
constexpr int NT = FMD_SMALL_NT;
constexpr int NW = NT / 64;
constexpr int TPX = 64;    // output pixels per tile
constexpr int LDS_MAX = 160 * 1024;

// n / d for 0 <= n < 2^31 by multiply-high (divisors fixed per launch, magic numbers made on the host)
struct FDiv {
  unsigned m;
  int s;
};
FDiv make_fdiv(unsigned d) {
  int s = 0;
  while ((1u << s) < d) ++s;
  return {(unsigned)(((1ull << 32) * ((1ull << s) - d)) / d + 1), s};
}
FMD_DEV int fdiv(int n, FDiv f) { return (int)((__umulhi((unsigned)n, f.m) + (unsigned)n) >> f.s); }

struct SArgs {
  fmd_conv_small_desc d;
  int C, T, HWs, HWo;
  int whole;        // tiles of whole images (Ho*Wo < 64)
  int S;            // images per tile (whole) else 1
  int trows;        // output rows per tile
  int tiles_per_n;  // pixel tiles per image (not whole)
  int ptiles, ctiles;
  int P, lgP;       // parts of the reduction (input channels) per tile (a power of two): one workgroup each
  int Cs;           // input channels per part (C / P)
  int in_rows;      // staged input rows per image
  int slots;        // staged pixel slots (the zero slot is index `slots`)
  int cmask;        // 16-byte-chunk swizzle mask
  int C23, C23s, cmask2;   // 1x1 segment channels (all, per part) and their swizzle mask
  int off_raw, off_ab, off_mr, off_gs, off_ep, off_st;   // LDS byte offsets (input region at 0)
  int cp;           // chunk parts (waves per row-block group)
  int gn;
  int bc;           // output channels per workgroup (16 or 32: the template instance)
  FDiv fd_c8, fd_rowslots, fd_ws, fd_c23, fd_hwo, fd_wo, fd_cg, fd_c2, fd_cs;   // fixed divisors (host magic)
  int cg_lanes;     // GroupNorm channels per group when a power of two <= 64 (the butterfly fold), else 0
  double inv_cnt;   // 1 / (channels per group x pixels per image)
  FDiv fd_pt;       // by ptiles
  int lnrb;         // log2 of the row blocks per wave
  int kw;           // 32-channel chunks per wave (the template instance, 1..4)
};

#ifdef FMD_SMALL_DBG
// ablation flags of a debug build (tools/build_variant.sh small -DFMD_SMALL_DBG; tools/small_abl.py):
// 1 no staging DMA, 2 no GroupNorm fold, 4 no main loop (weights, MFMAs), 8 no epilogue stores, 16 no statistics,
// 32 return at entry, 64 no raw / epilogue-operand / skip-weight loads, 128 the main loop twice
#define FMD_SMALL_TS
__device__ int g_small_dbg;
extern "C" int fmd_debug_small_flags(int f) { return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_small_dbg), &f, sizeof(int)); }
#define SDBG(bit) (g_small_dbg & (bit))
#else
#define SDBG(bit) false
#endif
#ifdef FMD_SMALL_TS
// phase timestamps (s_memrealtime, 100 MHz) of wave 0 of every workgroup: [block][12]; -DFMD_SMALL_TS alone adds
// only these (no flag loads, same register allocation as the product build, near enough)
constexpr int TS_MAX = 4096;
__device__ unsigned long long g_small_ts[TS_MAX * 12];
extern "C" int fmd_debug_small_ts(void* host, int nblocks, int clear) {
  if (clear) return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_small_ts), host, sizeof(unsigned long long) * 12 * nblocks);
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_small_ts), sizeof(unsigned long long) * 12 * nblocks);
}
#define STS(k)                                                                                      \
  do {                                                                                              \
    if (tid == 0 && blockIdx.x < TS_MAX) g_small_ts[blockIdx.x * 12 + (k)] = wall_clock64();       \
  } while (0)
#else
#define STS(k) do { } while (0)
#endif

FMD_DEV int swz(int c16, int slot, int cmask) { return (c16 & ~cmask) | ((c16 ^ slot) & cmask); }

typedef __attribute__((ext_vector_type(2))) int i32x2;
// a double from the lane DPP control CTRL names (both halves moved by v_mov_b32_dpp: no LDS round trip)
template <int CTRL>
FMD_DEV double dpp_d(double v) {
  const i32x2 x = __builtin_bit_cast(i32x2, v);
  i32x2 y;
  y.x = __builtin_amdgcn_update_dpp(0, x.x, CTRL, 0xF, 0xF, true);
  y.y = __builtin_amdgcn_update_dpp(0, x.y, CTRL, 0xF, 0xF, true);
  return __builtin_bit_cast(double, y);
}
// sum over aligned groups of g = 2^k <= 64 lanes, every lane of a group ends with the same value (the pairings are
// symmetric and fp addition commutes): quad xor 1, xor 2, row half-mirror, row mirror, then lane xor 16 / 32
FMD_DEV double group_sum(double v, int g) {
  if (g >= 2) v += dpp_d<0xB1>(v);    // quad_perm [1, 0, 3, 2]
  if (g >= 4) v += dpp_d<0x4E>(v);    // quad_perm [2, 3, 0, 1]
  if (g >= 8) v += dpp_d<0x141>(v);   // row_half_mirror
  if (g >= 16) v += dpp_d<0x140>(v);  // row_mirror
  if (g >= 32) {                      // ds_swizzle, bit mode: xor 16 within 32 lanes
    const i32x2 x = __builtin_bit_cast(i32x2, v);
    i32x2 y;
    y.x = __builtin_amdgcn_ds_swizzle(x.x, 0x401F);
    y.y = __builtin_amdgcn_ds_swizzle(x.y, 0x401F);
    v += __builtin_bit_cast(double, y);
  }
  if (g >= 64) v += __shfl_xor(v, 32, 64);
  return v;
}
// the same over aligned groups of 8 lanes, fp32
FMD_DEV float sum8(float v) {
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0xB1, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x4E, 0xF, 0xF, true));
  v += __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), 0x141, 0xF, 0xF, true));
  return v;
}

template <int BC, int KW>   // KW: 32-channel chunks per wave (plan), so only the fragments used are loaded
__global__ __launch_bounds__(NT, 512 / NT) void conv_small_kernel(const SArgs A) {
  constexpr int NCB = BC / 16;   // 16-cout MFMA blocks per wave
  extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
  const fmd_conv_small_desc& d = A.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int C = A.C, T = A.T, Cs = A.Cs;
  const int C8 = Cs >> 3;
  const int rowb = Cs * 2;   // bytes per LDS pixel row
  const unsigned lds0 = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)smem;
  STS(0);
  if (SDBG(32)) return;
  // Warm the scalar cache with every 64-byte line of the kernel arguments at once: the compiler loads each field
  // where it is first used, and each such cold load was a serial memory round trip (~1 us apiece, measured
  // with the phase timestamps of the FMD_SMALL_DBG build)
  {
    const __attribute__((address_space(4))) unsigned* ka =
        (const __attribute__((address_space(4))) unsigned*)__builtin_amdgcn_kernarg_segment_ptr();
    unsigned x = 0;
#pragma unroll
    for (int i = 0; i < (int)(sizeof(SArgs) + 63) / 64; ++i) x ^= ka[i * 16];
    asm volatile("; kernarg lines warm" ::"s"(x));
  }

  // block -> (tile, part): a tile's P parts are adjacent ids (one XCD after the remap); the cout tiles partition the
  // XCDs (each XCD's L2 holds its weight slice), the small input is shared
  const int nwg = A.ptiles * A.ctiles * A.P;
  const int bid = xcd_remap(blockIdx.x, nwg);
  const int kp = bid & (A.P - 1), tile = bid >> A.lgP;   // P: a power of two
  const int ct = fdiv(tile, A.fd_pt), pt = tile - ct * A.ptiles;
  const int k0 = ct * BC;
  const int cs0 = kp * Cs;   // this part's first input channel (of the virtual concat C0 | C1)

  int n0, oy0;
  if (A.whole) {
    n0 = pt * A.S;
    oy0 = 0;
  } else {
    n0 = pt / A.tiles_per_n;
    oy0 = (pt - n0 * A.tiles_per_n) * A.trows;
  }
  const int nS = A.whole ? min(A.S, d.N - n0) : 1;
  const int vpx = A.whole ? nS * A.HWo : TPX;
  int iy_lo = 0;
  if (!A.whole) iy_lo = d.mode == 0 ? oy0 - 1 : d.mode == 1 ? 2 * oy0 - 1 : d.mode == 2 ? (oy0 - 1) >> 1 : oy0;
  const size_t pix_base = A.whole ? (size_t)n0 * A.HWo : (size_t)n0 * A.HWo + (size_t)oy0 * d.Wo;

  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;
  const int C0 = d.C0, C1 = C - d.C0;
  const int rowslots = A.in_rows * d.Ws;
  const int units = nS * rowslots * C8;
  const int C23 = A.C23s, C238 = C23 >> 3;   // this part's 1x1-segment channels
  const int c2s0 = kp * C23;

  // The code runs once per workgroup (a few microseconds of work), so it is kept short -- loops, not unrolled
  // straight-line code that would be fetched cold by every workgroup -- and every global load is issued before the
  // first wait.

  // ---------------------------------------------------------------- (1) every weight fragment of this wave
  // wave (cp, rg): 32-channel chunks c = cp, cp + CP, ... (all taps of each), row blocks rg*NRB .. +NRB, all BC couts;
  // then the 1x1 segment's chunks cp, cp + CP, ...  All of its weight fragments (<= 36, plan) are loaded up front into
  // registers, so the MFMA loop never waits on memory: bq[(k*9 + t)*NCB + cb] (3x3), bq[k*NCB + cb] (1x1 main), the
  // skip chunks from bq[SKB + k*NCB + cb]
  const int CP = A.cp, RG = NW / CP, NRB = 4 / RG;
  const int cp = wid % CP, rg = wid / CP;
  const int nrbv = (vpx + 15) >> 4;    // row blocks holding valid pixels
  const int l16 = lane & 15, kq = lane >> 4;
  // Buffer loads, branch-free: a fragment past this wave's chunks gets an offset beyond the descriptor's range (the
  // load returns zeros without touching memory).  A per-fragment "if (valid) load" made hipcc branch around every
  // load and put an s_waitcnt vmcnt(0) in front of each -- a serial chain of memory round trips.
  constexpr unsigned OOR = 0x80000000u;
  const int nch = SDBG(4) ? 0 : Cs >> 5;
  const bool keep_raw = C23 > 0;
  const int nch2 = C23 >> 5;
  bf16x8 bq[KW * 9 * NCB];   // 3x3: [k][tap][cb]; 1x1: the first KW * NCB as [k][cb]
  bf16x8 bs[4 * NCB];        // the 1x1 segment's [k][cb]
  {
    const auto rw = __builtin_amdgcn_make_buffer_rsrc((void*)d.wgt, 0, d.K * T * C * 2, 0x00020000);
    const unsigned wl = (unsigned)(((k0 + l16) * T * C + cs0 + kq * 8) * 2);   // this lane's row, bytes
    const unsigned wcb = 16u * T * C * 2;                                       // between the 16-cout blocks
    if (T == 9) {
#pragma unroll
      for (int k = 0; k < KW; ++k)
#pragma unroll
        for (int t = 0; t < 9; ++t)
#pragma unroll
          for (int cb = 0; cb < NCB; ++cb) {
            const int c = cp + k * CP;
            const unsigned off = c < nch ? wl + cb * wcb + (unsigned)(t * C + c * 32) * 2 : OOR;
            bq[(k * 9 + t) * NCB + cb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0));
          }
    } else {
#pragma unroll
      for (int k = 0; k < KW; ++k)
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) {
          const int c = cp + k * CP;
          const unsigned off = c < nch ? wl + cb * wcb + (unsigned)(c * 32) * 2 : OOR;
          bq[k * NCB + cb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw, off, 0, 0));
        }
    }
  }
  if (keep_raw && !SDBG(64)) {
    const auto rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)d.wgt2, 0, d.K * A.C23 * 2, 0x00020000);
    const unsigned wl2 = (unsigned)(((k0 + l16) * A.C23 + c2s0 + kq * 8) * 2);
#pragma unroll
    for (int k = 0; k < 4; ++k)
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) {
        const int c = cp + k * CP;
        const unsigned off = c < nch2 ? wl2 + (unsigned)(cb * 16 * A.C23 + c * 32) * 2 : OOR;
        bs[k * NCB + cb] = __builtin_bit_cast(bf16x8, __builtin_amdgcn_raw_buffer_load_b128(rw2, off, 0, 0));
      }
  }

  STS(10);
  // ---------------------------------------------------------------- (2) everything else global -> LDS by DMA
  // Input region: LDS unit q (16 bytes) is physical chunk u of slot q / C8, which holds logical chunk swz(u, slot)
  // (the swizzle is an involution); padding rows get zeros by ds_write.  Then the raw 1x1-segment input of the tile's
  // output pixels; then the GroupNorm inputs (the tile's statistics slab rows of this part's channels, gamma, beta,
  // the scale-shift rows).  All of it is in flight together (asm DMAs, not tracked by hipcc: the vmcnt(0) below).
  for (int q0 = wid * 64; q0 < units; q0 += NT) {
    if (SDBG(1)) break;
    const int q = q0 + lane;
    if (q < units) {
      const int slot = fdiv(q, A.fd_c8), c = cs0 + swz(q - slot * C8, slot, A.cmask) * 8;
      // whole images: the slots are the tile's pixels in order, no padding rows
      int iy = 0;
      size_t gp = (size_t)n0 * A.HWs + slot;
      if (!A.whole) {
        const int r = fdiv(slot, A.fd_ws), ix = slot - r * d.Ws;
        iy = iy_lo + r;
        gp = ((size_t)n0 * d.Hs + iy) * d.Ws + ix;
      }
      if (iy >= 0 && iy < d.Hs) {
        glds16(c < C0 ? s0 + gp * C0 + c : s1 + gp * C1 + (c - C0), __builtin_amdgcn_readfirstlane(lds0 + q0 * 16));
      } else {
        *(u32x4*)(smem + q * 16) = u32x4{0u, 0u, 0u, 0u};
      }
    }
  }
  const int uraw = SDBG(64) ? 0 : vpx * C238;
  for (int q0 = wid * 64; q0 < uraw; q0 += NT) {
    const int q = q0 + lane;
    if (q < uraw) {
      const int p = fdiv(q, A.fd_c23), c = c2s0 + swz(q - p * C238, p, A.cmask2) * 8;
      const size_t gp = pix_base + p;
      glds16(c < d.C2 ? (const bf16r*)d.src2 + gp * d.C2 + c : (const bf16r*)d.src3 + gp * d.C3 + (c - d.C2),
             __builtin_amdgcn_readfirstlane(lds0 + A.off_raw + q0 * 16));
    }
  }
  for (int c8 = tid; c8 < C8; c8 += NT) *(u32x4*)(smem + A.slots * rowb + c8 * 16) = u32x4{0u, 0u, 0u, 0u};
  // this part's channels [cs0, cs0 + Cs) in the two sources: src0 channels [a0, a0 + m0), src1 channels [a1, a1 + m1)
  const int a0 = min(cs0, C0), m0 = min(cs0 + Cs, C0) - a0;
  const int a1 = max(cs0, C0) - C0, m1 = Cs - m0;
  const int E0 = A.gn ? A.HWs / d.rows0 : 0, E1 = A.gn && C1 ? A.HWs / d.rows1 : 0;
  float* gs = (float*)(smem + A.off_gs);                  // [nS][E0][m0][2] | [nS][E1][m1][2] | gamma | beta | emb
  float* gs1 = gs + (size_t)nS * E0 * m0 * 2;
  float* gam = gs1 + (size_t)nS * E1 * m1 * 2;
  float* bet = gam + Cs;
  float* emb = bet + Cs;                                  // [nS][2][Cs] (scale, shift)
  if (A.gn && !SDBG(2)) {
#pragma unroll
    for (int src = 0; src < 2; ++src) {   // per slab row (image, pixel block): m channels x (sum, sum of squares)
      const int m = src ? m1 : m0, E = src ? E1 : E0, Cx = src ? C1 : C0, ax = src ? a1 : a0;
      const int h = m >> 1;                // 16-byte units per row
      const int n16 = nS * E * h;
      const float* st = (src ? d.st1 : d.st0) + ((size_t)n0 * E * Cx + ax) * 2;
      const unsigned dst = lds0 + A.off_gs + (src ? (unsigned)((char*)gs1 - (char*)gs) : 0u);
      for (int q0 = wid * 64; q0 < n16; q0 += NT) {
        const int q = q0 + lane;
        if (q < n16) {
          const int row = q / h;
          glds16(st + ((size_t)row * Cx + (q - row * h) * 2) * 2, __builtin_amdgcn_readfirstlane(dst + q0 * 16));
        }
      }
    }
    const unsigned dg = lds0 + A.off_gs + (unsigned)((char*)gam - (char*)gs);
    for (int q0 = wid * 64; q0 < Cs; q0 += NT)
      if (q0 + lane < Cs) {
        if (d.gamma) glds4(d.gamma + cs0 + q0 + lane, __builtin_amdgcn_readfirstlane(dg + q0 * 4));
        else gam[q0 + lane] = 1.f;
        if (d.beta) glds4(d.beta + cs0 + q0 + lane, __builtin_amdgcn_readfirstlane(dg + (Cs + q0) * 4));
        else bet[q0 + lane] = 0.f;
      }
    if (d.emb)
      for (int q0 = wid * 64; q0 < nS * 2 * Cs; q0 += NT) {
        const int q = q0 + lane;
        if (q < nS * 2 * Cs) {
          const int si = fdiv(q, A.fd_c2), rem = q - si * 2 * Cs, hs = rem >= Cs;
          glds4(d.emb + (size_t)(n0 + si) * d.emb_stride + hs * C + cs0 + (rem - hs * Cs),
                __builtin_amdgcn_readfirstlane(dg + (2 * Cs + q0) * 4));
        }
      }
  }
  STS(1);
  // epilogue operands of the tile: bias, skip bias, the images' per-sample bias rows (BC floats each) and the
  // residual tile (bf16 [pixel][BC]); absent ones are zeros.  In LDS, not registers: the main loop needs those.
  float* eb = (float*)(smem + A.off_ep);                  // [2 + nS][BC]
  bf16r* er = (bf16r*)(smem + A.off_ep + (2 + A.S) * BC * 4);   // [TPX][BC]
  {
    const int KS = d.bias_nc_stride ? d.bias_nc_stride : d.K;
    const int ne = (2 + nS) * BC;
    for (int q0 = wid * 64; q0 < ne; q0 += NT) {
      const int q = q0 + lane;
      if (q < ne) {
        const int r = q / BC, j = q - r * BC;
        const float* src = r == 0 ? d.bias : r == 1 ? d.bias2 : d.bias_nc ? d.bias_nc + (size_t)(n0 + r - 2) * KS : nullptr;
        if (src && !SDBG(64)) glds4(src + k0 + j, __builtin_amdgcn_readfirstlane(lds0 + A.off_ep + q0 * 4));
        else eb[q] = 0.f;
      }
    }
    const int nr = vpx * (BC / 8);
    for (int q0 = wid * 64; q0 < nr; q0 += NT) {
      const int q = q0 + lane;
      if (q < nr) {
        const int pp = q / (BC / 8), j = q - pp * (BC / 8);
        if (d.resid && !SDBG(64))
          glds16((const bf16r*)d.resid + (pix_base + pp) * d.K + k0 + j * 8,
                 __builtin_amdgcn_readfirstlane(lds0 + (unsigned)((char*)er - (char*)smem) + q0 * 16));
        else
          *(u32x4*)(er + q * 8) = u32x4{0u, 0u, 0u, 0u};
      }
    }
  }
  // The main loop's LDS addresses, one table for the workgroup: stab[pixel][tap] = the byte offset of the tap's input
  // row (or the zero slot's), with the slot's low swizzle bits (sl & cmask) * 16 in the low bits -- rowb is a
  // multiple of 16 * (cmask + 1), so they are free -- and a fragment address is (sb ^ (c16 & cmask) * 16) +
  // (c16 & ~cmask) * 16.  Each thread fills one or two of the TPX x 9 entries (pure ALU, while the loads above are
  // in flight) instead of every lane computing its own 36.
  int* stab = (int*)(smem + A.off_st);   // [TPX][12]
  {
    const int sm = d.mode == 1 ? 2 : 1, shf = d.mode == 2 ? 1 : 0;
    const int Hl = d.mode == 2 ? d.Ho : d.Hs, Wl = d.mode == 2 ? d.Wo : d.Ws;
    const int zsb = A.slots * rowb + (A.slots & A.cmask) * 16;
    for (int e = tid; e < TPX * 9; e += NT) {
      const int p = e / 9, t = e - p * 9;
      const int s = A.whole ? fdiv(p, A.fd_hwo) : 0;
      const int rem = A.whole ? p - s * A.HWo : oy0 * d.Wo + p;
      const int oy = fdiv(rem, A.fd_wo), ox = rem - oy * d.Wo;
      const int ky = T == 1 ? 1 : t / 3, kx = T == 1 ? 1 : t - (t / 3) * 3;
      const int yy = oy * sm + ky - 1, xx = ox * sm + kx - 1;
      const int sl = (s * A.in_rows - iy_lo + (yy >> shf)) * d.Ws + (xx >> shf);
      const bool ok = p < vpx && t < T && yy >= 0 && yy < Hl && xx >= 0 && xx < Wl;
      stab[p * 12 + t] = ok ? sl * rowb + (sl & A.cmask) * 16 : zsb;
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // this wave's DMAs have landed
  __syncthreads();
  STS(2);

  // ---------------------------------------------------------------- (3) GroupNorm affine, from LDS
  float2* ab = (float2*)(smem + A.off_ab);   // [nS][Cs]: channel totals (sum, sum of squares), then (a, b)
  float2* mr = (float2*)(smem + A.off_mr);   // [nS][Cs / Cg] (mean, rstd)
  if (A.gn && !SDBG(2) && A.cg_lanes) {
    // Groups of Cg = 2^k <= 64 channels: thread i holds channel i of [nS][Cs] (a group's channels are consecutive
    // lanes of one wave), sums its slab rows, the group totals meet by an fp64 butterfly over the Cg lanes, and every
    // lane forms its own (a, b) -- no serial per-group loop, one barrier
    const int Cg = A.cg_lanes;
    const double inv_cnt = A.inv_cnt;
    for (int i0 = 0; i0 < nS * Cs; i0 += NT) {   // the same trip count in every wave: the shuffles see whole groups
      const int i = i0 + tid;
      const bool act = i < nS * Cs;
      const int si = act ? fdiv(i, A.fd_cs) : 0, cl = act ? i - si * Cs : 0;
      const bool in0 = cl < m0;
      const int E = act ? (in0 ? E0 : E1) : 0, m = in0 ? m0 : m1;
      const float2* p = (const float2*)(in0 ? gs : gs1) + ((size_t)si * E * m + (in0 ? cl : cl - m0));
      float2 f0 = make_float2(0.f, 0.f), f1 = make_float2(0.f, 0.f);
      int e = 0;
      for (; e + 1 < E; e += 2) {
        const float2 x0 = p[(size_t)e * m], x1 = p[(size_t)(e + 1) * m];
        f0.x += x0.x; f0.y += x0.y; f1.x += x1.x; f1.y += x1.y;
      }
      if (e < E) { const float2 x0 = p[(size_t)e * m]; f0.x += x0.x; f0.y += x0.y; }
      const double t1 = group_sum((double)(f0.x + f1.x), Cg), t2 = group_sum((double)(f0.y + f1.y), Cg);
      if (act) {
        const double mean = t1 * inv_cnt;
        double var = t2 * inv_cnt - mean * mean;
        if (var < 0) var = 0;
        const float mf = (float)mean, rs = rsqrtf((float)var + d.eps);
        float a = rs * gam[cl];
        float b = bet[cl] - mf * a;
        if (d.emb) {
          const float sc = 1.f + emb[si * 2 * Cs + cl];
          a *= sc;
          b = b * sc + emb[si * 2 * Cs + Cs + cl];
        }
        ab[i] = make_float2(a, b);
      }
    }
    __syncthreads();
  } else if (A.gn && !SDBG(2)) {
    for (int i = tid; i < nS * Cs; i += NT) {
      const int si = i / Cs, cl = i - si * Cs;
      const bool in0 = cl < m0;
      const int E = in0 ? E0 : E1, m = in0 ? m0 : m1;
      const float2* p = (const float2*)(in0 ? gs : gs1) + ((size_t)si * E * m + (in0 ? cl : cl - m0));
      float2 t0 = make_float2(0.f, 0.f), t1 = make_float2(0.f, 0.f);
      int e = 0;
      for (; e + 1 < E; e += 2) {
        const float2 x0 = p[(size_t)e * m], x1 = p[(size_t)(e + 1) * m];
        t0.x += x0.x; t0.y += x0.y; t1.x += x1.x; t1.y += x1.y;
      }
      if (e < E) { const float2 x0 = p[(size_t)e * m]; t0.x += x0.x; t0.y += x0.y; }
      ab[i] = make_float2(t0.x + t1.x, t0.y + t1.y);
    }
    __syncthreads();
    const int Cg = C / d.G, Gs = Cs / Cg;
    for (int i = tid; i < nS * Gs; i += NT) {
      const int si = i / Gs, g = i - si * Gs;
      double t1 = 0.0, t2 = 0.0;
      for (int j = 0; j < Cg; ++j) {
        const float2 t = ab[si * Cs + g * Cg + j];
        t1 += t.x;
        t2 += t.y;
      }
      const double cnt = (double)Cg * A.HWs;
      const double mean = t1 / cnt;
      double var = t2 / cnt - mean * mean;
      if (var < 0) var = 0;
      mr[i] = make_float2((float)mean, (float)(1.0 / sqrt(var + (double)d.eps)));
    }
    __syncthreads();
    for (int i = tid; i < nS * Cs; i += NT) {
      const int si = i / Cs, cl = i - si * Cs;
      const float2 m = mr[si * Gs + fdiv(cl, A.fd_cg)];
      float a = m.y * gam[cl];
      float b = bet[cl] - m.x * a;
      if (d.emb) {
        const float sc = 1.f + emb[si * 2 * Cs + cl];
        a *= sc;
        b = b * sc + emb[si * 2 * Cs + Cs + cl];
      }
      ab[i] = make_float2(a, b);
    }
    __syncthreads();
  }

  STS(11);
  // ---------------------------------------------------------------- (4) GroupNorm affine + SiLU, in place in LDS
  if (A.gn) {
    for (int q = tid; q < units; q += NT) {
      const int slot = fdiv(q, A.fd_c8), c8 = swz(q - slot * C8, slot, A.cmask);
      const int s = A.whole ? fdiv(slot, A.fd_rowslots) : 0;
      if (!A.whole) {
        const int iy = iy_lo + fdiv(slot, A.fd_ws);
        if (iy < 0 || iy >= d.Hs) continue;   // padding stays zero
      }
      u32x4 w = *(const u32x4*)(smem + q * 16);
      const float4* abp = (const float4*)(ab + s * Cs + c8 * 8);
      float y[8];
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const float4 qq = abp[h];
        y[2 * h] = bf_lo(w[h]) * qq.x + qq.y;
        y[2 * h + 1] = bf_hi(w[h]) * qq.z + qq.w;
      }
      if (d.silu) {
#pragma unroll
        for (int e = 0; e < 8; ++e) y[e] = siluf_(y[e]);
      }
#pragma unroll
      for (int h = 0; h < 4; ++h) w[h] = pack2(y[2 * h], y[2 * h + 1]);
      *(u32x4*)(smem + q * 16) = w;
    }
    __syncthreads();
  }

  STS(3);
  // ---------------------------------------------------------------- (5) epilogue unit of this thread
  const bool has_eu = tid < vpx * (BC / 8);     // (pixel, 8-cout group)
  const int ep = tid / (BC / 8), ej = tid % (BC / 8);
  const int eco = k0 + ej * 8;

  // ---------------------------------------------------------------- (6) main loop
  // per (row block, tap): the LDS byte offset of this lane's pixel row (or the zero slot's), with the slot's low
  // swizzle bits (sl & cmask) * 16 in the low bits -- rowb is a multiple of 16 * (cmask + 1), so they are free -- and
  // a fragment address is (sb ^ (c16 & cmask) * 16) + (c16 & ~cmask) * 16

  const int c16m_mask = A.cmask;
  int slotv[4][9];
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r >= NRB) continue;
    const int4* q = (const int4*)(stab + ((rg * NRB + r) * 16 + l16) * 12);
    const int4 v0 = q[0], v1 = q[1];
    slotv[r][0] = v0.x; slotv[r][1] = v0.y; slotv[r][2] = v0.z; slotv[r][3] = v0.w;
    slotv[r][4] = v1.x; slotv[r][5] = v1.y; slotv[r][6] = v1.z; slotv[r][7] = v1.w;
    slotv[r][8] = stab[((rg * NRB + r) * 16 + l16) * 12 + 8];
  }
  f32x4 acc[4][NCB];
#pragma unroll
  for (int r = 0; r < 4; ++r)
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) acc[r][cb] = f32x4{0.f, 0.f, 0.f, 0.f};
  // one step: the tap's pixel fragments of this wave's row blocks x the NCB weight fragments bq[b .. b + NCB)
  auto step = [&](int b, int c32, int t) {
    const int c16 = c32 * 4 + kq;
    const int lo = (c16 & c16m_mask) * 16, hi = (c16 & ~c16m_mask) * 16;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      if (r >= NRB || (rg * NRB + r) >= nrbv) continue;
      const bf16x8 bfr = *(const bf16x8*)(smem + ((slotv[r][t] ^ lo) + hi));
#pragma unroll
      for (int cb = 0; cb < NCB; ++cb) acc[r][cb] = mfma16(bq[b + cb], bfr, acc[r][cb]);
    }
  };
#ifdef FMD_SMALL_DBG
  // flag 128: the main loop twice (timing only: the second pass runs with a warm instruction cache)
  for (int rep = 0; rep < (SDBG(128) ? 2 : 1); ++rep) {
    if (rep == 1) STS(8);
#endif
  if (T == 9) {
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int c = cp + k * CP;
      if (c >= nch) break;
#pragma unroll
      for (int t = 0; t < 9; ++t) step((k * 9 + t) * NCB, c, t);
    }
  } else {
#pragma unroll
    for (int k = 0; k < KW; ++k) {
      const int c = cp + k * CP;
      if (c >= nch) break;
      step(k * NCB, c, 0);
    }
  }
#ifdef FMD_SMALL_DBG
    if (rep == 1) STS(9);
  }
#endif
  // 1x1 segment over the raw sources at the tile's pixels (ResBlock skip conv)
  if (keep_raw) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const int c = cp + k * CP;
      if (c >= nch2) break;
      const int c16 = c * 4 + kq;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (r >= NRB || (rg * NRB + r) >= nrbv) continue;
        const int p = (rg * NRB + r) * 16 + l16;
        const bf16x8 bfr = *(const bf16x8*)(smem + A.off_raw + p * (C23 * 2) + swz(c16, p, A.cmask2) * 16);
#pragma unroll
        for (int cb = 0; cb < NCB; ++cb) acc[r][cb] = mfma16(bs[k * NCB + cb], bfr, acc[r][cb]);
      }
    }
  }
  STS(4);
  __syncthreads();   // every wave is done with the staged input: its LDS becomes the combine scratch
  STS(5);

  // ---------------------------------------------------------------- (7) combine + epilogue
  // red[wave][pixel][cout]: lane (l16 = pixel, kq = 4-cout group) holds couts 4 kq .. 4 kq + 3 of its pixel
  float* red = (float*)smem;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    if (r >= NRB) continue;
    const int p = (rg * NRB + r) * 16 + l16;
#pragma unroll
    for (int cb = 0; cb < NCB; ++cb) *(f32x4*)(red + ((size_t)wid * TPX + p) * BC + cb * 16 + kq * 4) = acc[r][cb];
  }
  __syncthreads();
  const int g = (ep >> 4) >> A.lnrb;   // row-block group: the waves g*CP .. g*CP + CP - 1 hold this pixel
  f32x4 o0 = f32x4{0.f, 0.f, 0.f, 0.f}, o1 = f32x4{0.f, 0.f, 0.f, 0.f};
  if (has_eu) {
    for (int q = 0; q < CP; ++q) {
      const float* src = red + ((size_t)(g * CP + q) * TPX + ep) * BC + ej * 8;
      o0 += *(const f32x4*)src;
      o1 += *(const f32x4*)(src + 4);
    }
  }
  if (A.P > 1) {
    // Combine of the P parts inside the launch (MI355X_MICROARCH.md, inter-workgroup visibility: a counter hand-off
    // with write-through payload).  Every part stores its partial tile to its slot of the tile's slab with sc1 stores,
    // every wave drains them, then ONE lane takes a ticket (relaxed agent-scope add); the part drawing P - 1 is the
    // reducer: it resets the ticket for the next launch and reads all P slots with sc1 loads, in part order (the sum
    // does not depend on which part arrives last).
    const int slab_b = A.P * TPX * BC * 4;
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(d.part + (size_t)tile * A.P * TPX * BC, 0, slab_b, 0x00020000);
    const int eoff = (ep * BC + ej * 8) * 4;
    if (has_eu) {
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o0), rsrc, kp * TPX * BC * 4 + eoff, 0, 16);
      __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, o1), rsrc, kp * TPX * BC * 4 + eoff + 16, 0, 16);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* last = (int*)(smem + A.off_ab);   // outside the combine scratch
    if (tid == 0) {
      auto* tk = (__attribute__((address_space(1))) unsigned*)(d.tickets + tile);
      const unsigned t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = t == (unsigned)(A.P - 1);
      if (is_last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = is_last;
    }
    __syncthreads();
    STS(6);
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (has_eu) {
      // all 16 slots' loads in flight at once: past the P parts the descriptor's range check returns zeros
      u32x4 v[16][2];
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        v[q][0] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, q * TPX * BC * 4 + eoff, 0, 16);
        v[q][1] = __builtin_amdgcn_raw_buffer_load_b128(rsrc, q * TPX * BC * 4 + eoff + 16, 0, 16);
      }
      o0 = f32x4{0.f, 0.f, 0.f, 0.f};
      o1 = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int q = 0; q < 16; ++q) {
        o0 += __builtin_bit_cast(f32x4, v[q][0]);
        o1 += __builtin_bit_cast(f32x4, v[q][1]);
      }
    }
  }
  if (has_eu) {
    const int si = A.whole ? fdiv(ep, A.fd_hwo) : 0;
    const float* b0 = eb + ej * 8;
    const float* b1 = eb + BC + ej * 8;
    const float* b2 = eb + (2 + si) * BC + ej * 8;
    const u32x4 erv = *(const u32x4*)(er + ep * BC + ej * 8);
    float o[8] = {o0[0], o0[1], o0[2], o0[3], o1[0], o1[1], o1[2], o1[3]};
#pragma unroll
    for (int e = 0; e < 8; ++e) o[e] += b0[e] + b1[e] + b2[e];
#pragma unroll
    for (int h = 0; h < 4; ++h) { o[2 * h] += bf_lo(erv[h]); o[2 * h + 1] += bf_hi(erv[h]); }
    u32x4 w;
#pragma unroll
    for (int h = 0; h < 4; ++h) w[h] = pack2(o[2 * h], o[2 * h + 1]);
    if (!SDBG(8)) *(u32x4*)((bf16r*)d.out + (pix_base + ep) * d.K + eco) = w;
    // the statistics are taken on the rounded values the consumer reads (over this pixel's first slice)
    float* dst = red + ((size_t)(g * CP) * TPX + ep) * BC + ej * 8;
#pragma unroll
    for (int h = 0; h < 4; ++h) { dst[2 * h] = bf_lo(w[h]); dst[2 * h + 1] = bf_hi(w[h]); }
  }
  STS(7);
  if (!d.stats || SDBG(16)) return;
  __syncthreads();
  // (row, cout) sums over the row's pixels: 8 lanes per (row, cout), each summing every 8th pixel, then a fixed
  // butterfly over the 8 lanes (deterministic).  One slab row per image (whole tiles) or per 64-pixel tile.
  const int nrows = A.whole ? nS : 1, rpx = A.whole ? A.HWo : TPX;
  for (int u0 = 0; u0 < nrows * BC * 8; u0 += NT) {
    const int u = u0 + tid;
    const int part = u & 7, rc = u >> 3;
    const int row = rc / BC, co = rc - row * BC;
    float t1 = 0.f, t2 = 0.f;
    if (row < nrows) {
      for (int i = part; i < rpx; i += 8) {
        const int p = row * rpx + i;
        const float x = red[((size_t)(((p >> 4) >> A.lnrb) * CP) * TPX + p) * BC + co];
        t1 += x;
        t2 += x * x;
      }
    }
    t1 = sum8(t1);
    t2 = sum8(t2);
    if (part == 0 && row < nrows) {
      const size_t grow = A.whole ? (size_t)(n0 + row) : (size_t)n0 * A.tiles_per_n + (oy0 / A.trows);
      d.stats[(grow * d.K + k0 + co) * 2] = t1;
      d.stats[(grow * d.K + k0 + co) * 2 + 1] = t2;
    }
  }
}

#ifndef FMD_SMALL_SPLIT_WG
#define FMD_SMALL_SPLIT_WG 256
#endif
constexpr int SPLIT_WG = FMD_SMALL_SPLIT_WG;   // automatic split: parts until the launch has this many workgroups

int plan(const fmd_conv_small_desc* d, SArgs* A) {
  if (!d || d->N < 1 || d->K < 16 || !d->src0 || !d->wgt || !d->out) return -1;
  const int C = d->C0 + d->C1;
  if (d->C0 % 8 || d->C1 % 8 || (d->C1 && !d->src1) || C % 32 || C < 64) return -2;
  switch (d->mode) {
    case 0: case 3: if (d->Ho != d->Hs || d->Wo != d->Ws) return -3; break;
    case 1: if (d->Hs != 2 * d->Ho || d->Ws != 2 * d->Wo) return -3; break;
    case 2: if (d->Ho != 2 * d->Hs || d->Wo != 2 * d->Ws) return -3; break;
    default: return -3;
  }
  const int C23 = d->C2 > 0 ? d->C2 + d->C3 : 0;
  if (C23 && (C23 % 32 || d->C2 % 8 || d->C3 % 8 || (d->C3 && !d->src3) || !d->src2 || !d->wgt2 ||
              (d->mode != 0 && d->mode != 3)))
    return -4;
  const bool gn = d->st0 != nullptr;
  if (gn && (d->G < 1 || C % d->G || d->rows0 < 1 || (d->C1 && (!d->st1 || d->rows1 < 1)))) return -5;
  if (d->split < 0 || d->split > 16 || (d->split & (d->split - 1))) return -8;
  A->d = *d;
  A->C = C;
  A->T = d->mode == 3 ? 1 : 9;
  A->HWs = d->Hs * d->Ws;
  A->HWo = d->Ho * d->Wo;
  if (gn && (A->HWs % d->rows0 || (d->C1 && A->HWs % d->rows1))) return -5;
  if (A->HWo >= TPX) {
    if (A->HWo % TPX || TPX % d->Wo) return -6;
    A->whole = 0;
    A->S = 1;
    A->trows = TPX / d->Wo;
    A->tiles_per_n = d->Ho / A->trows;
    A->ptiles = d->N * A->tiles_per_n;
    A->in_rows = d->mode == 0 ? A->trows + 2 : d->mode == 1 ? 2 * A->trows + 1 : d->mode == 2 ? A->trows / 2 + 2
                                                                                              : A->trows;
  } else {
    if (TPX % A->HWo) return -6;
    A->whole = 1;
    A->S = d->N < TPX / A->HWo ? d->N : TPX / A->HWo;
    A->trows = d->Ho;
    A->tiles_per_n = 1;
    A->in_rows = d->Hs;
  }
  if (d->K % 16) return -1;
  const int Cg = gn ? C / d->G : 1;
  const int E0 = gn ? A->HWs / d->rows0 : 0, E1 = gn && d->C1 ? A->HWs / d->rows1 : 0;
  // a split of the reduction into P parts: 32-channel chunks, at least two per part, whole groups, and the 1x1
  // segment split alike
  auto part_ok = [&](int P) {
    const int cs = C / P;
    return C % P == 0 && cs % 32 == 0 && cs >= 64 && (!gn || cs % Cg == 0) && (!C23 || (C23 % P == 0 && (C23 / P) % 32 == 0));
  };
  // every weight fragment of a wave in 36 registers: main chunks per wave <= 4 / NCB (3x3) or 36 / NCB (1x1), the
  // 1x1 segment's <= 4, and together within 36
  auto frag_ok = [&](int bc, int P) {
    const int nch = C / P / 32, cp = nch >= NW ? NW : nch >= 4 ? 4 : 2;
    const int ncb = bc / 16, kw = (nch + cp - 1) / cp, kw2 = (C23 / P / 32 + cp - 1) / cp;
    const int mainf = kw * A->T * ncb;
    // instances: 16 couts x 1..4 chunks per wave, 32 couts x 1 chunk (more would spill)
    return !(kw2 > 4 || kw > (bc == 32 ? 1 : 4) || mainf > 36 || (C23 && mainf > 36 - 4 * ncb));
  };
  for (;;) {   // fewer images per tile until the LDS plan fits
    if (A->whole) A->ptiles = (d->N + A->S - 1) / A->S;
    // 32 output channels per workgroup (half the redundant staging per channel) only where that still fills the chip
    // unsplit; else 16, which halves the parts the reduction needs (the split's ticket and combine cost a workgroup
    // ~2.5 us; config D's 16^2 level: 15.9 us at 32 couts x 2 parts)
    int bc = d->K % 32 == 0 && A->ptiles * (d->K / 32) >= SPLIT_WG ? 32 : 16;
    int P = 1;
    for (;;) {
      const int nwg1 = A->ptiles * (d->K / bc);
      const bool ws = d->part && d->tickets && d->n_tickets >= nwg1;
      auto fits = [&](int p) { return (long long)nwg1 * p * TPX * bc * 4 <= d->part_bytes; };
      if (d->split > 1) {
        if (!ws || !part_ok(d->split) || !fits(d->split)) return -8;
        P = d->split;
      } else if (d->split == 0 && ws) {
        P = 1;
        while (nwg1 * P < SPLIT_WG && P < 16 && part_ok(2 * P) && fits(2 * P)) P *= 2;
        while (!frag_ok(bc, P) && P < 16 && part_ok(2 * P) && fits(2 * P)) P *= 2;   // fewer fragments per part
      }
      if (frag_ok(bc, P)) break;
      if (bc == 32) { bc = 16; continue; }   // 16-cout workgroups: half the fragments per wave
      return -4;
    }
    A->bc = bc;
    A->P = P;
    A->Cs = C / P;
    A->C23 = C23;
    A->C23s = C23 / P;
    const int Cs = A->Cs;
    A->slots = A->S * A->in_rows * d->Ws;
    const int tpx = A->whole ? A->S * A->HWo : TPX;
    const int in_b = (A->slots + 1) * Cs * 2;
    const int raw_b = tpx * A->C23s * 2;
    const int red_b = NW * TPX * A->bc * 4;
    const int body = in_b + raw_b > red_b ? in_b + raw_b : red_b;
    A->off_raw = in_b;
    A->off_ab = (body + 15) / 16 * 16;
    A->off_mr = A->off_ab + (gn && A->S * Cs * 8 > 16 ? A->S * Cs * 8 : 16);   // >= 16: the reducer's flag word
    A->off_gs = (A->off_mr + (gn ? A->S * (Cs / Cg) * 8 : 0) + 15) / 16 * 16;
    // + the GroupNorm inputs: slab rows of this part's channels (at most Cs of one source per row), gamma, beta,
    // scale-shift rows
    const int Emax = E0 > E1 ? E0 : E1;
    const int gs_b = gn ? A->S * Emax * Cs * 8 + 2 * Cs * 4 + (d->emb ? A->S * 2 * Cs * 4 : 0) : 0;
    A->off_ep = (A->off_gs + gs_b + 15) / 16 * 16;
    // + the epilogue operands: bias, skip bias, per-sample bias rows, the residual tile
    A->off_st = A->off_ep + (2 + A->S) * bc * 4 + TPX * bc * 2;
    // + the main loop's address table [TPX][12] ints
    const int total = A->off_st + TPX * 12 * 4;
    if (total <= LDS_MAX && (!gn || A->S * Cs <= 8192)) {
      A->ctiles = d->K / A->bc;
      const int c8 = Cs / 8;
      A->cmask = c8 % 16 == 0 ? 15 : c8 % 8 == 0 ? 7 : c8 % 4 == 0 ? 3 : 1;
      const int c238 = A->C23s / 8;
      A->cmask2 = c238 % 16 == 0 ? 15 : c238 % 8 == 0 ? 7 : c238 % 4 == 0 ? 3 : 1;
      A->fd_c23 = make_fdiv(c238 > 0 ? c238 : 1);
      const int nch = Cs / 32;
      A->cp = nch >= NW ? NW : nch >= 4 ? 4 : 2;
      A->kw = (nch + A->cp - 1) / A->cp;
      A->gn = gn;
      A->fd_c8 = make_fdiv(c8);
      A->fd_rowslots = make_fdiv(A->in_rows * d->Ws);
      A->fd_ws = make_fdiv(d->Ws);
      A->fd_hwo = make_fdiv(A->HWo);
      A->fd_wo = make_fdiv(d->Wo);
      A->fd_cg = make_fdiv(Cg);
      A->fd_c2 = make_fdiv(2 * Cs);
      A->fd_cs = make_fdiv(Cs);
      A->cg_lanes = gn && Cg <= 64 && (Cg & (Cg - 1)) == 0 ? Cg : 0;
      A->inv_cnt = 1.0 / ((double)Cg * A->HWs);
      A->fd_pt = make_fdiv(A->ptiles);
      A->lgP = 0;
      while ((1 << A->lgP) < A->P) ++A->lgP;
      const int nrb = 4 * A->cp / NW;                  // NRB = 4 / (NW / cp)
      A->lnrb = nrb == 4 ? 2 : nrb == 2 ? 1 : 0;
      return total;
    }
    if (!A->whole || A->S == 1) return -7;
    A->S /= 2;
  }
}

}  // namespace

extern "C" int fmd_conv_small_plan(const fmd_conv_small_desc* d) {
  SArgs A;
  return plan(d, &A);
}

extern "C" int fmd_conv_small_split(const fmd_conv_small_desc* d) {
  SArgs A;
  const int r = plan(d, &A);
  return r < 0 ? r : A.P;
}

template <int BC, int KW>
const void* kfn() { return (const void*)conv_small_kernel<BC, KW>; }

extern "C" int fmd_conv_small(const fmd_conv_small_desc* d, fmd_stream_t s) {
  SArgs A;
  const int lds = plan(d, &A);
  if (lds < 0) return lds;
  static const void* const fns[5] = {kfn<16, 1>(), kfn<16, 2>(), kfn<16, 3>(), kfn<16, 4>(), kfn<32, 1>()};
  static bool attr = false;
  if (!attr) {
    for (const void* f : fns) {
      const hipError_t e = hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_MAX);
      if (e != hipSuccess) return (int)e;
    }
    attr = true;
  }
  if (A.kw < 1 || A.kw > 4 || (A.bc == 32 && A.kw != 1)) return -9;   // the plan allows no other instance
  const void* f = fns[A.bc == 32 ? 4 : A.kw - 1];
  void* args[] = {&A};
  const hipError_t e = hipLaunchKernel(f, dim3(A.ptiles * A.ctiles * A.P), dim3(NT), args, lds, (hipStream_t)s);
  if (e != hipSuccess) return (int)e;
  return (int)hipGetLastError();
}
