// Halo-tiled 3x3 stride-1 convolution, v10: producer / consumer waves in a persistent workgroup.
//
// Why: in v9b every wave both staged the GN+SiLU halo (VALU, transcendentals), ran the MFMAs and
// did its tile's epilogue, and the two co-resident workgroups of a CU ran those phases in lock-step, so the VALU of
// one wave sat behind the MFMAs of its SIMD partner and the MFMA pipe idled through prologues / epilogues (PMC:
// MFMA busy 45 %, 5.9 non-MFMA VALU per MFMA; the kernel without MFMAs still took 70-80 % of its time).
//
// v10 gives each role its own waves.  One 512-thread workgroup per CU (persistent over the tiles lb, lb + G, ...):
//   * waves 0-3, consumers (s_setprio 1): the v9b main loop -- one 32-cout quarter of the 16x16-pixel x 128-cout tile
//     per wave, 8 accumulators of v_mfma_f32_32x32x16_bf16, A fragments from the staged halo, B fragments straight
//     from L2 two taps ahead -- and a short epilogue: residual / SiLU' side values brought into the accumulator layout
//     by identity MFMAs, bf16 pack, transpose back to channels-last by permuted-identity MFMAs into the LDS out tile;
//   * waves 4-7, producers (priority 0): stage the NEXT chunk's halo (global loads one chunk ahead, GN affine + SiLU,
//     zero padding) into the other halo buffer, store the PREVIOUS tile's output from the LDS out tile with its
//     per-64-pixel GroupNorm statistics, and fill the out tile with the CURRENT tile's side values (residual copy, or
//     the data gradient's SiLU'(ep_a x + ep_b) in fp16) before its epilogue.
// Producer wave w owns the tile's pixels [64w, 64w + 64) (= statistics row w) for its store and side-fill jobs, so a
// wave only ever re-writes out-tile bytes it has itself read.  One s_barrier per chunk orders everything:
//   interval g (consumers run global chunk g of this workgroup from halo buffer g & 1):
//     producers: halo(g + 1) -> buffer (g + 1) & 1; loads of chunk g + 2; at the tile's chunk 1: store(tile - 1),
//                side(tile) first half; at chunk 2 (or 1): side(tile) second half
//     consumers: 9 taps (or one 1x1 tap of the skip segment); after a tile's last chunk: epilogue into the out tile
// The epilogue of tile t lies between the barrier ending t's last chunk and the one ending t+1's chunk 0, so the
// store at t+1's chunk 1 reads a finished tile; tiles need >= 2 chunks (3x3 + 1x1), else v9b runs the problem.
//
// Same operand layouts and pre-tiled weights as v9b (csrc/conv_halo9.hip); no split-K (the small levels keep v9b's
// split path), no nearest-x2 gather, no stride-2 modes, no G side output.
#include "halo_args.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
typedef __attribute__((ext_vector_type(2))) float f32x2;
typedef __attribute__((ext_vector_type(2))) _Float16 f16x2;

constexpr int NT10 = 512, NPT = 256;             // threads; producer threads
constexpr int TH = 16, TW = 16, BCO = 128, BK = 32, KC = BK / 8;
constexpr int WTILE = KC * BCO * 16;             // bytes of one tap's weight tile (8 KiB)
constexpr int HROW = TW + 2, HPOS = (TH + 2) * HROW;
constexpr int HPOSP = (HPOS + 7) / 8 * 8;
constexpr int HPAD = (HPOSP + 15) / 16 * 16;     // plane stride == 0 mod 16 bank slots
constexpr int HBUF = KC * HPAD * 16;             // bytes per halo buffer
constexpr int NR = (HPOSP * KC + NPT - 1) / NPT; // staging rounds per 3x3 chunk (6)
constexpr int OUTB = TH * TW * BCO * 2;          // out / side tile (64 KiB, 16-byte pieces XOR-swizzled per pixel)
constexpr int SM_OUT = 2 * HBUF;
constexpr int SM_BYTES = SM_OUT + OUTB;
constexpr int ZFLAG = 1 << 30;                   // staged piece: store zeros (padding / invalid channels)
static_assert(NR <= 6, "staging rounds");
static_assert(SM_BYTES <= 160 * 1024, "LDS");
// debug ablations (A.dbg via fmd_debug_halo_flags; compiled in only with -DFMD_HALO_DBG, tools/build_variant.sh):
// 1 producers skip halo staging, 2 producers skip store / side jobs, 4 consumers skip MFMAs, 8 consumers skip B
// loads, 16 consumers skip the epilogue
#ifdef FMD_HALO_DBG
#define HDBG10(bit) (A.dbg & (bit))
#else
#define HDBG10(bit) false
#endif
// phase timeline (-DFMD_HALO_TIME; tools/h10_timeline.py): lane 0 of wave 0 (consumer) and wave 4 (producer) stamp
// s_memtime at fixed points of every chunk interval into A.tbuf[block][2][H10_NS]
constexpr int H10_NS = 512;
#ifdef FMD_HALO_TIME
#define HT10(role, idx)                                                                                  \
  do {                                                                                                   \
    if ((wid == 0 || wid == 4) && lane == 0 && (idx) < H10_NS) {                                         \
      unsigned long long t_;                                                                             \
      asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t_)::"memory");                         \
      A.tbuf[((size_t)blockIdx.x * 2 + (role)) * H10_NS + (idx)] = t_;                                    \
    }                                                                                                    \
  } while (0)
#else
#define HT10(role, idx) do {} while (0)
#endif
#ifndef FMD_H10_PIN
#define FMD_H10_PIN 1
#endif

FMD_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}
FMD_DEV f32x16 mfma32h(const f16x8& a, const f16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_f16(a, b, c, 0, 0, 0);
}
FMD_DEV bf16x8 as_bf16x8(const u32x4& u) { return __builtin_bit_cast(bf16x8, u); }
FMD_DEV unsigned packh(float lo, float hi) {   // RNE fp32 pair -> fp16 pair (v_cvt_pk_f16_f32)
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2{lo, hi}, f16x2));
}
// chunk boundary: this wave's LDS writes done, then the workgroup barrier.  Raw s_barrier: vector-memory loads stay
// in flight across it (producers' next-chunk loads, consumers' B fragments two taps ahead)
FMD_DEV void wg_barrier() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}
FMD_DEV void set_prio(int p) {   // wave priority (s_setprio takes an immediate)
  if (p == 3) __builtin_amdgcn_s_setprio(3);
  else if (p == 2) __builtin_amdgcn_s_setprio(2);
  else if (p == 1) __builtin_amdgcn_s_setprio(1);
  else __builtin_amdgcn_s_setprio(0);
}
// register fence over 16 values: all are materialised here, before any later instruction reads them
FMD_DEV void fence16(float (&y)[16]) {
  asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]),
               "+v"(y[8]), "+v"(y[9]), "+v"(y[10]), "+v"(y[11]), "+v"(y[12]), "+v"(y[13]), "+v"(y[14]), "+v"(y[15]));
}
FMD_DEV void fence8(float (&y)[8]) {
  asm volatile("" : "+v"(y[0]), "+v"(y[1]), "+v"(y[2]), "+v"(y[3]), "+v"(y[4]), "+v"(y[5]), "+v"(y[6]), "+v"(y[7]));
}
// 16-byte piece (pixel p, channel octet o) of the out / side tile: XOR swizzle over the 16 octets of a pixel row
FMD_DEV int tile_off(int p, int o) { return p * 256 + ((o ^ (p & 15)) << 4); }

struct Tile {
  int tco, ptile, n, smp, zz, ty0, tx0;
};
FMD_DEV Tile tile_of(const HArgs& A, int t) {
  Tile T;
  T.tco = t % A.ntc;
  T.ptile = t / A.ntc;
  const int per = A.tiles_x * A.tiles_y;
  T.n = T.ptile / per;
  const int tin = T.ptile - T.n * per;
  T.smp = A.depth ? T.n / A.depth : T.n;
  T.zz = A.depth ? T.n - T.smp * A.depth : 0;
  const int tyi = tin / A.tiles_x;
  T.ty0 = tyi * TH;
  T.tx0 = (tin - tyi * A.tiles_x) * TW;
  return T;
}
FMD_DEV int opix_of(const fmd_conv_desc& d, const Tile& T, int pi) {
  return (T.n * d.Ho + T.ty0 + (pi >> 4)) * d.Wo + T.tx0 + (pi & 15);
}

// PRO: 0 raw input, 1 GroupNorm affine, 2 affine + SiLU.  SIDE: 0 none, 1 residual, 2 data-gradient SiLU'.
template <int PRO, int SIDE>
__global__ __launch_bounds__(NT10) __attribute__((amdgpu_waves_per_eu(2, 2)))
void conv3x3_halo10(const HArgs A, int ntiles, int prio) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_BYTES];
  unsigned char* const tileb = smem + SM_OUT;
  const fmd_conv_desc& d = A.d;
  const int tid = threadIdx.x, wid = tid >> 6, lane = tid & 63;
  const int G = gridDim.x;
  const int lb = xcd_remap(blockIdx.x, G);
  const int nt = (ntiles - lb + G - 1) / G;      // tiles lb, lb + G, ... (>= 1: G <= ntiles)
  const int nch = A.nchunk1 + A.nchunk2;         // chunks per tile (>= 2)
  const int total = nt * nch;
  const int K = d.K;

  if (wid < 4) {
    // ============================================================== consumers
    set_prio(prio & 3);
    const int r = lane & 31, hh = lane >> 5, rr = r >> 4;
    const int col = rr ? ((r - 18) & 15) : r;
    const int abase = (hh * HPAD + rr * HROW + col) * 16;
    const int boff = (hh * BCO + 32 * wid + r) * 16;
    const int T1 = A.nchunk1 * 9;
    const int S = T1 + A.nchunk2;                 // weight slots per tile
    const unsigned char* const wt1 = (const unsigned char*)A.wt;
    const unsigned char* const wt2 = (const unsigned char*)A.wt2;
    // B fragments: slot sl of tile it (3x3 taps 0 .. T1-1, then the 1x1 chunks) -> its 8 KiB tile; loads run two
    // slots ahead.  Slots past the last tile map to a valid one (loaded, never consumed)
    auto slot_ptr = [&](int it_, int sl_) -> const unsigned char* {
      it_ += sl_ / S;
      sl_ %= S;
      if (it_ >= nt) {
        it_ = nt - 1;
        sl_ = S - 1;
      }
      const int tco = (lb + it_ * G) % A.ntc;
      return sl_ < T1 ? wt1 + ((size_t)tco * T1 + sl_) * WTILE : wt2 + ((size_t)tco * A.nchunk2 + (sl_ - T1)) * WTILE;
    };
    auto loadB = [&](bf16x8 (&bq)[2], const unsigned char* base) {
      if (!HDBG10(8)) {
        bq[0] = *(const bf16x8*)(base + boff);
        bq[1] = *(const bf16x8*)(base + boff + 4096);
      }
    };
    f32x16 acc[8];
    bf16x8 bq_[3][2];
    auto init_acc = [&](int it) {
      const Tile T = tile_of(A, lb + it * G);
      const int co = T.tco * BCO + 32 * wid + r;
      float bsum = 0.f;
      if (d.bias) bsum += d.bias[co];
      if (d.bias2) bsum += d.bias2[co];
      if (d.bias_nc) bsum += d.bias_nc[(size_t)T.smp * K + co];
#pragma unroll
      for (int pb = 0; pb < 8; ++pb)
#pragma unroll
        for (int e = 0; e < 16; ++e) acc[pb][e] = bsum;
    };
    auto aoff = [&](int tap, int s, int pb) {
      const int ky = tap / 3, kx = tap % 3;
      return abase + (s * 2 * HPAD + (2 * pb + ky) * HROW + kx) * 16;
    };
    // one tap: 8 pixel blocks x 2 k-steps = 16 MFMAs, the 16 A-fragment reads four groups ahead (as v9b)
    auto tap_mma = [&](int tap, int hb, const bf16x8 (&bq)[2]) {
      if (HDBG10(4)) return;
      bf16x8 af[16];
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) af[4 * g + i] = *(const bf16x8*)(smem + hb + aoff(tap, g >> 1, 4 * (g & 1) + i));
#pragma unroll
      for (int g = 0; g < 4; ++g)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[4 * (g & 1) + i] = mfma32(af[4 * g + i], bq[g >> 1], acc[4 * (g & 1) + i]);
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x100, 4, 0);
      __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);
    };
    // one 3x3 chunk: 144 MFMAs (9 taps x 2 k-steps x 8 pixel blocks) in one stream whose A fragments are read 8
    // MFMAs ahead through a 16-entry register ring, across tap boundaries: with one consumer wave per SIMD nothing
    // else hides an LDS read, so only the chunk's first 8 reads (after its barrier) are exposed.  MFMA f: tap
    // f >> 4, k-step (f >> 3) & 1, pixel block f & 7 (the same accumulator recurs 8 MFMAs later)
    auto chunk_mma = [&](int hb, const unsigned char* wc, const unsigned char* nx0, const unsigned char* nx1) {
      if (HDBG10(4)) {
#pragma unroll
        for (int t = 0; t < 9; ++t) loadB(bq_[(t + 2) % 3], t < 7 ? wc + (t + 2) * WTILE : t == 7 ? nx0 : nx1);
        return;
      }
      // per-tap laundered LDS bases: taps (ky, pb) and (ky + 2, pb - 1) read the same fragment, and hipcc would
      // otherwise keep such fragments live across taps (CSE) and spill
      int tb[9];
#pragma unroll
      for (int t = 0; t < 9; ++t) {
        tb[t] = hb;
        asm volatile("" : "+v"(tb[t]));
      }
      bf16x8 af[16];
#pragma unroll
      for (int f = 0; f < 8; ++f) af[f] = *(const bf16x8*)(smem + tb[0] + aoff(0, f >> 3, f & 7));
#pragma unroll
      for (int tap = 0; tap < 9; ++tap) {
        loadB(bq_[(tap + 2) % 3], tap < 7 ? wc + (tap + 2) * WTILE : tap == 7 ? nx0 : nx1);
#pragma unroll
        for (int w = 0; w < 16; ++w) {
          const int fn = tap * 16 + w + 8;   // the read 8 MFMAs ahead
          if (fn < 144) af[(w + 8) & 15] = *(const bf16x8*)(smem + tb[fn >> 4] + aoff(fn >> 4, (fn >> 3) & 1, fn & 7));
          acc[w & 7] = mfma32(af[w], bq_[tap % 3][w >> 3], acc[w & 7]);
        }
      }
      // pin the interleave: 8 reads, then per MFMA one read ahead (+ the tap's two B loads at its start)
#if FMD_H10_PIN  // pinned read / MFMA interleave (default on; -DFMD_H10_PIN=0 for the compiler's own schedule)
      __builtin_amdgcn_sched_group_barrier(0x100, 8, 0);
#pragma unroll
      for (int f = 0; f < 144; ++f) {
        if ((f & 15) == 0) __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);
        if (f + 8 < 144) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
#endif
    };
    // identity B operands: inat brings a channels-last 32-channel slice into the accumulator layout, iperm
    // transposes a packed accumulator back (v9b epilogue)
    // epilogue: identity B operands (inat brings a channels-last 32-channel slice into the accumulator layout, iperm
    // transposes a packed accumulator back; v9b), built per tile so they hold no registers through the main loop
    const int cl = 32 * wid;
    auto epilogue = [&]() {
      if (HDBG10(16)) return;
      bf16x8 inat[2], iperm[2];
      f16x8 inath[2];
#pragma unroll
      for (int s = 0; s < 2; ++s)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          inat[s][j] = (__bf16)((16 * s + 8 * hh + j) == r ? 1.0f : 0.0f);
          inath[s][j] = (_Float16)((16 * s + 8 * hh + j) == r ? 1.0f : 0.0f);
          iperm[s][j] = (__bf16)((16 * s + 8 * (j >> 2) + 4 * hh + (j & 3)) == r ? 1.0f : 0.0f);
        }
#pragma unroll
      for (int pb = 0; pb < 8; ++pb) {
        const int q = r >> 4;
        const int pi_l = (2 * pb + q) * TW + (q ? ((r - 18) & 15) : r);
        f32x16 v = acc[pb];
        if (SIDE) {
          u32x4 fr[2];
#pragma unroll
          for (int s = 0; s < 2; ++s) fr[s] = *(const u32x4*)(tileb + tile_off(pi_l, (cl + 16 * s + 8 * hh) >> 3));
          if (SIDE == 1) {   // residual: added exactly in fp32
#pragma unroll
            for (int s = 0; s < 2; ++s) v = mfma32(as_bf16x8(fr[s]), inat[s], v);
          } else {           // SiLU'(ep_a x + ep_b) in fp16
            f32x16 xc;
#pragma unroll
            for (int e = 0; e < 16; ++e) xc[e] = 0.f;
#pragma unroll
            for (int s = 0; s < 2; ++s) xc = mfma32h(__builtin_bit_cast(f16x8, fr[s]), inath[s], xc);
#pragma unroll
            for (int e = 0; e < 16; ++e) v[e] *= xc[e];
          }
        }
        bf16x8 pf[2];
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          u32x4 u;
#pragma unroll
          for (int e = 0; e < 4; ++e) u[e] = pack2(v[8 * s + 2 * e], v[8 * s + 2 * e + 1]);
          pf[s] = as_bf16x8(u);
        }
        f32x16 z;
#pragma unroll
        for (int e = 0; e < 16; ++e) z[e] = 0.f;
#pragma unroll
        for (int s = 0; s < 2; ++s) z = mfma32(pf[s], iperm[s], z);
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          u32x2 o;
          o[0] = pack2(z[4 * g], z[4 * g + 1]);
          o[1] = pack2(z[4 * g + 2], z[4 * g + 3]);
          *(u32x2*)(tileb + tile_off(pi_l, 4 * wid + g) + 8 * hh) = o;
        }
      }
    };

    auto& bq = bq_;
    loadB(bq[0], slot_ptr(0, 0));
    loadB(bq[1], slot_ptr(0, 1));
    init_acc(0);
    wg_barrier();   // B0: chunk 0 staged
    int g = 0;
    for (int it = 0; it < nt; ++it) {
      for (int cc = 0; cc < A.nchunk1; ++cc, ++g) {
        const int s0 = cc * 9;
        HT10(0, 4 * g);
        chunk_mma((g & 1) * HBUF, slot_ptr(it, s0), slot_ptr(it, s0 + 9), slot_ptr(it, s0 + 10));
        HT10(0, 4 * g + 1);
        wg_barrier();
      }
      // 1x1 skip segment: one (centre) tap per chunk; the ring unrolled by 3 so no copy waits on a load in flight
      for (int i = 0; i < A.nchunk2; i += 3) {
#pragma unroll
        for (int k = 0; k < 3; ++k) {
          if (i + k < A.nchunk2) {
            loadB(bq[(k + 2) % 3], slot_ptr(it, T1 + i + k + 2));
            tap_mma(4, (g & 1) * HBUF, bq[k]);
            wg_barrier();
            ++g;
          }
        }
      }
      if (A.nchunk2 % 3) {   // back to the 3x3 chunks' ring phase (slot s in bq[0], s + 1 in bq[1])
        const int ph = A.nchunk2 % 3;
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          const bf16x8 b0 = bq[0][h], b1 = bq[1][h], b2 = bq[2][h];
          bq[0][h] = ph == 1 ? b1 : b2;
          bq[1][h] = ph == 1 ? b2 : b0;
        }
      }
      HT10(0, 4 * (g - 1) + 2);
      epilogue();
      HT10(0, 4 * (g - 1) + 3);
      if (it + 1 < nt) init_acc(it + 1);
    }
    wg_barrier();   // B_end: the last epilogue is in the out tile
    return;
  }

  // ================================================================ producers
  set_prio((prio >> 2) & 3);
  const int pt = tid - NPT, pw = wid - 4;
  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;
  const bf16r* __restrict__ s2 = (const bf16r*)d.src2;
  const bf16r* __restrict__ s3 = (const bf16r*)d.src3;
  const int kc = (pt >> 3) & (KC - 1);
  const int p0 = (pt >> 5) * 8 + (pt & 7);
  const int sdst0 = (kc * HPAD + p0) * 16;
  const int s2dst0 = (kc * HPAD + ((p0 >> 4) + 1) * HROW + (p0 & 15) + 1) * 16;
  const int sdummy = (kc * HPAD + HPOS) * 16;   // a slot of the plane no tap reads (HPOS < HPAD)
  const unsigned HWs = (unsigned)(d.Hs * d.Ws);

  // ---- halo staging.  Geometry of the tile whose chunks are being loaded (recomputed once per tile): the halo
  // pixel (y * Ws + x) of each round's piece, -1 for padding, and its LDS slot
  int st_it = -1, st_n = 0, st_smp = 0, st_zz = 0, s2pix0 = 0;
  int spx[NR], sdst[NR];
  auto stage_geom = [&](int it) {
    const Tile T = tile_of(A, lb + it * G);
    st_it = it;
    st_n = T.n;
    st_smp = T.smp;
    st_zz = T.zz;
#pragma unroll
    for (int q = 0; q < NR; ++q) {
      const int pos = q * 64 + p0;
      const int py = pos / HROW, px = pos - py * HROW;
      const int y = T.ty0 - 1 + py, x = T.tx0 - 1 + px;
      spx[q] = (pos < HPOS && y >= 0 && y < d.Hs && x >= 0 && x < d.Ws) ? y * d.Ws + x : -1;
      sdst[q] = pos < HPOS ? sdst0 + q * 1024 : sdummy;
    }
    s2pix0 = (T.n * d.Ho + T.ty0 + (p0 >> 4)) * d.Wo + T.tx0 + (p0 & 15);
  };
  // the chunk in flight: raw pieces, their LDS slots, zero-store mask, GN affine of this thread's channel octet
  u32x4 rh[NR];
  int cdst[NR];
  unsigned zm = 0;
  float qa[8], qb[8];
  bool xf = false;
  int it_ld = 0, cc_ld = 0;   // next chunk to load
  // per-lane (VGPR) copies of the staging arguments: left uniform, hipcc re-loads them from the kernel arguments
  // inside the loop (scalar loads + waits on the producer's path)
  unsigned long long g_s0 = (unsigned long long)s0, g_s1 = (unsigned long long)(s1 ? s1 : s0);
  unsigned long long g_s2 = (unsigned long long)(s2 ? s2 : s0), g_s3 = s3 ? (unsigned long long)s3 : g_s2;
  unsigned long long g_pa = (unsigned long long)d.pro_a, g_pb = (unsigned long long)d.pro_b;
  int v_C0 = d.C0, v_C1 = d.C1, v_C2 = d.C2, v_C3 = d.C3, v_C = A.C, v_C23 = A.C23, v_Wo = d.Wo;
  asm volatile("" : "+v"(g_s0), "+v"(g_s1), "+v"(g_s2), "+v"(g_s3), "+v"(g_pa), "+v"(g_pb));
  asm volatile("" : "+v"(v_C0), "+v"(v_C1), "+v"(v_C2), "+v"(v_C3), "+v"(v_C), "+v"(v_C23), "+v"(v_Wo));
  auto issue = [&]() {   // loads of the next chunk (it_ld, cc_ld): branch-free per-lane address arithmetic
    if (HDBG10(1)) return;
    if (it_ld != st_it) stage_geom(it_ld);
    const int cc = cc_ld;
    zm = 0;
    if (cc < A.nchunk1) {
      int cb = cc, sl = st_n;
      bool zok = true;
      if (A.depth) {
        const int kz = cc / A.ncb;
        cb = cc - kz * A.ncb;
        const int zl = st_zz + kz - 1;
        zok = zl >= 0 && zl < A.depth;
        sl = st_smp * A.dsrc + zl;
      }
      const int c = cb * BK + kc * 8;
      const bool in0 = c < v_C0;
      const int scs = in0 ? v_C0 : v_C1;
      const bool sok = c < v_C && zok;
      const unsigned long long gb = in0 ? g_s0 : g_s1;
      // element offset of (slice sl, pixel 0, this lane's channel octet); the launcher keeps it below 2^31
      const unsigned el0 = (unsigned)(sl * (int)HWs) * (unsigned)scs + (unsigned)(in0 ? c : c - v_C0);
      if (PRO != 0) {
        const unsigned long long co = (unsigned long long)(st_smp * v_C + (sok ? c : 0)) * 4;
        const f32x4 a0 = *(const f32x4*)(g_pa + co), a1 = *(const f32x4*)(g_pa + co + 16);
        const f32x4 b0 = *(const f32x4*)(g_pb + co), b1 = *(const f32x4*)(g_pb + co + 16);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          qa[e] = a0[e]; qa[4 + e] = a1[e];
          qb[e] = b0[e]; qb[4 + e] = b1[e];
        }
      }
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        const bool valid = sok && spx[q] >= 0;
        const unsigned el = el0 + __umul24((unsigned)spx[q], (unsigned)scs);
        rh[q] = *(const u32x4*)(valid ? gb + (unsigned long long)el * 2 : g_s0);
        zm |= valid ? 0u : (1u << q);
        cdst[q] = sdst[q];
      }
      xf = PRO != 0;
    } else {
      const int c = (cc - A.nchunk1) * BK + kc * 8;
      const bool in2 = c < v_C2;
      const bool sok = c < v_C23;
      const int scs = in2 ? v_C2 : v_C3;
      const unsigned long long gb = in2 ? g_s2 : g_s3;
      const unsigned el0 = (unsigned)s2pix0 * (unsigned)scs + (unsigned)(in2 ? c : c - v_C2);
#pragma unroll
      for (int q = 0; q < NR; ++q) {
        if (q < 4) {
          const unsigned el = el0 + (unsigned)(4 * q * v_Wo) * (unsigned)scs;
          rh[q] = *(const u32x4*)(sok ? gb + (unsigned long long)el * 2 : g_s0);
          cdst[q] = s2dst0 + q * 72 * 16;
        } else {
          cdst[q] = sdummy;
        }
        zm |= (sok && q < 4) ? 0u : (1u << q);
      }
      xf = false;
    }
    if (++cc_ld == nch) {
      cc_ld = 0;
      ++it_ld;
    }
  };
  // transform + store the chunk in flight into halo buffer byte offset buf (no branches).  The GN affine + SiLU of
  // two pieces (16 elements) advance stage by stage behind register fences: a single producer wave per SIMD issues
  // in order, and the compiler's element-by-element chains (fma -> mul -> exp -> add -> rcp -> mul) left it
  // waiting out each dependent result (~80 ticks per element, tools/h10_timeline.py)
  auto commit = [&](int buf) {
    if (HDBG10(1)) return;
#pragma unroll
    for (int qp = 0; qp < NR; qp += 2) {
      u32x4 v[2] = {rh[qp], rh[qp + 1]};
      if (PRO != 0 && xf) {
        float y[16], t[16];
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            y[8 * k + 2 * e] = bf_lo(v[k][e]);
            y[8 * k + 2 * e + 1] = bf_hi(v[k][e]);
          }
        fence16(y);
#pragma unroll
        for (int j = 0; j < 16; ++j) y[j] = y[j] * qa[j & 7] + qb[j & 7];
        fence16(y);
        if (PRO == 2) {
#pragma unroll
          for (int j = 0; j < 16; ++j) t[j] = y[j] * -1.4426950408889634f;
          fence16(t);
#pragma unroll
          for (int j = 0; j < 16; ++j) t[j] = __builtin_amdgcn_exp2f(t[j]);
          fence16(t);
#pragma unroll
          for (int j = 0; j < 16; ++j) t[j] = 1.f + t[j];
          fence16(t);
#pragma unroll
          for (int j = 0; j < 16; ++j) t[j] = __builtin_amdgcn_rcpf(t[j]);
          fence16(t);
#pragma unroll
          for (int j = 0; j < 16; ++j) y[j] = y[j] * t[j];
        }
#pragma unroll
        for (int k = 0; k < 2; ++k)
#pragma unroll
          for (int e = 0; e < 4; ++e) v[k][e] = pack2(y[8 * k + 2 * e], y[8 * k + 2 * e + 1]);
      }
#pragma unroll
      for (int k = 0; k < 2; ++k) {
        const bool z = (zm >> (qp + k)) & 1u;
#pragma unroll
        for (int e = 0; e < 4; ++e) v[k][e] = z ? 0u : v[k][e];
        *(u32x4*)(smem + buf + cdst[qp + k]) = v[k];
      }
    }
  };

  // ---- tile jobs.  Unit u of tile it: u < 4 stores tile row 4 pw + u of tile it - 1 from the out tile (16 pixels x
  // the lane's channel octet: pixel column 4 j + ps, j = 0..3) with its GroupNorm statistics; u >= 4 (SIDE) fills
  // row 4 pw + u - 4 of the out tile with tile it's side values.  Units run in order over the tile's chunk
  // intervals 1 .. nch-1 (a side row after the store of the same row); a unit's global loads (the previous tile's x
  // for the data-gradient statistics, the residual / x side data) are issued at the end of the interval before.
  const int o = lane & 15, ps = lane >> 4;
  const bool stats = d.stats != nullptr;
  const bool hasx = d.ep_x0 != nullptr;
  const int NU = SIDE ? 8 : 4;
  auto unit_iv = [&](int u) { return 1 + (u * (nch - 1)) / NU; };
  constexpr int MAXU = 3;        // prefetch slots (units per interval beyond these load in place)
  u32x4 ub[MAXU][4];
  float st1[8], st2[8];
  Tile Tp, Tc;                   // job geometry: tile it - 1 (stores) and tile it (side)
  auto rowpix = [&](const Tile& T, int row) { return (T.n * d.Ho + T.ty0 + 4 * pw + row) * d.Wo + T.tx0 + ps; };
  auto xptr = [&](int gp, int c) -> const u32x4* {   // data-gradient side input x at (pixel gp, channel c)
    return (const u32x4*)((c < d.ep_C0) ? (const bf16r*)d.ep_x0 + (size_t)gp * d.ep_C0 + c
                                        : (const bf16r*)d.ep_x1 + (size_t)gp * (K - d.ep_C0) + (c - d.ep_C0));
  };
  auto unit_load = [&](int it, int u, u32x4 (&dst)[4]) {
    if (u < 4) {
      if (!(stats && hasx) || it == 0) return;
      const int c = Tp.tco * BCO + 8 * o, gp0 = rowpix(Tp, u);
#pragma unroll
      for (int j = 0; j < 4; ++j) dst[j] = *xptr(gp0 + 4 * j, c);
    } else {
      const int c = Tc.tco * BCO + 8 * o, gp0 = rowpix(Tc, u - 4);
#pragma unroll
      for (int j = 0; j < 4; ++j)
        dst[j] = SIDE == 1 ? *(const u32x4*)((const bf16r*)d.resid + (size_t)(gp0 + 4 * j) * K + c) : *xptr(gp0 + 4 * j, c);
    }
  };
  auto unit_run = [&](int it, int u, const u32x4 (&src)[4]) {
    if (u < 4) {
      if (it == 0) return;
      const int c = Tp.tco * BCO + 8 * o, gp0 = rowpix(Tp, u);
      if (u == 0) {
#pragma unroll
        for (int e = 0; e < 8; ++e) { st1[e] = 0.f; st2[e] = 0.f; }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int p = 64 * pw + 16 * u + 4 * j + ps;
        const u32x4 w = *(const u32x4*)(tileb + tile_off(p, o));
        *(u32x4*)((bf16r*)d.out + (size_t)(gp0 + 4 * j) * K + c) = w;
        const u32x4 xv = hasx ? src[j] : w;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const float w0 = bf_lo(w[e]), w1 = bf_hi(w[e]);
          st1[2 * e] += w0;
          st1[2 * e + 1] += w1;
          st2[2 * e] += w0 * bf_lo(xv[e]);
          st2[2 * e + 1] += w1 * bf_hi(xv[e]);
        }
      }
      if (u == 3 && stats) {   // statistics row pw: sum the 4 pixel-column lanes (ps) of each octet, fixed order
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          const auto a1 = __builtin_amdgcn_permlane32_swap(__float_as_uint(st1[e]), __float_as_uint(st1[e]), false, false);
          const auto a2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(st2[e]), __float_as_uint(st2[e]), false, false);
          const float t1 = __uint_as_float(a1[0]) + __uint_as_float(a1[1]);
          const float t2 = __uint_as_float(a2[0]) + __uint_as_float(a2[1]);
          const auto b1 = __builtin_amdgcn_permlane16_swap(__float_as_uint(t1), __float_as_uint(t1), false, false);
          const auto b2 = __builtin_amdgcn_permlane16_swap(__float_as_uint(t2), __float_as_uint(t2), false, false);
          st1[e] = __uint_as_float(b1[0]) + __uint_as_float(b1[1]);
          st2[e] = __uint_as_float(b2[0]) + __uint_as_float(b2[1]);
        }
        if (ps == 0) {
          float* sp = d.stats + ((size_t)(Tp.ptile * 4 + pw) * K + c) * 2;
#pragma unroll
          for (int e = 0; e < 4; ++e)
            *(f32x4*)(sp + 4 * e) = f32x4{st1[2 * e], st2[2 * e], st1[2 * e + 1], st2[2 * e + 1]};
        }
      }
    } else if (SIDE) {
      const int c = Tc.tco * BCO + 8 * o;
      float ea[8], eb[8];
      if (SIDE == 2) {
        const float* pa = d.ep_a + (size_t)Tc.smp * K + c;
        const float* pbp = d.ep_b + (size_t)Tc.smp * K + c;
        const f32x4 a0 = *(const f32x4*)pa, a1 = *(const f32x4*)(pa + 4);
        const f32x4 b0 = *(const f32x4*)pbp, b1 = *(const f32x4*)(pbp + 4);
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          ea[e] = a0[e]; ea[4 + e] = a1[e];
          eb[e] = b0[e]; eb[4 + e] = b1[e];
        }
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {   // one piece (8 elements) per staged pass
        u32x4 v = src[j];
        if (SIDE == 2) {   // SiLU'(z) = s (1 + z (1 - s)), s = 1 / (1 + exp(-z)), z = ep_a x + ep_b
          float z[8], t[8];
#pragma unroll
          for (int e = 0; e < 4; ++e) {
            z[2 * e] = ea[2 * e] * bf_lo(v[e]) + eb[2 * e];
            z[2 * e + 1] = ea[2 * e + 1] * bf_hi(v[e]) + eb[2 * e + 1];
          }
          fence8(z);
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = z[i] * -1.4426950408889634f;
          fence8(t);
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_exp2f(t[i]);
          fence8(t);
#pragma unroll
          for (int i = 0; i < 8; ++i) t[i] = __builtin_amdgcn_rcpf(1.f + t[i]);
          fence8(t);
#pragma unroll
          for (int i = 0; i < 8; ++i) z[i] = t[i] * (z[i] * (1.f - t[i]) + 1.f);
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = packh(z[2 * e], z[2 * e + 1]);
        }
        *(u32x4*)(tileb + tile_off(64 * pw + 16 * (u - 4) + 4 * j + ps, o)) = v;
      }
    }
  };
  // interval cc of tile it: run the units scheduled there, then prefetch those of interval cc + 1.  Units of one
  // interval are consecutive, so slot u % MAXU is free of collisions while an interval holds <= MAXU units (nch >= 4
  // with side jobs, nch >= 3 without); otherwise every unit loads in place
  const bool pref = (NU + nch - 2) / (nch - 1) <= MAXU;
  auto jobs = [&](int it, int cc) {
    if (HDBG10(2)) return;
    if (cc == 0) {
      if (it > 0) Tp = Tc;
      Tc = tile_of(A, lb + it * G);
    }
#pragma unroll
    for (int u = 0; u < NU; ++u) {
      if (unit_iv(u) != cc) continue;
      if (pref) {
        unit_run(it, u, ub[u % MAXU]);
      } else {
        u32x4 tmp[4];
        unit_load(it, u, tmp);
        unit_run(it, u, tmp);
      }
    }
    if (pref) {
#pragma unroll
      for (int u = 0; u < NU; ++u)
        if (unit_iv(u) == cc + 1) unit_load(it, u, ub[u % MAXU]);
    }
  };

  issue();
  commit(0);
  if (total > 1) issue();
  wg_barrier();   // B0
  int it = 0, cc = 0;
  for (int g = 0; g < total; ++g) {
    HT10(1, 4 * g);
#ifdef FMD_HALO_TIME
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // time build only: separates the load wait from the transform
    HT10(1, 256 + g);
#endif
    if (g + 1 < total) commit(((g + 1) & 1) * HBUF);
    HT10(1, 4 * g + 1);
    if (g + 2 < total) issue();
    HT10(1, 4 * g + 2);
    jobs(it, cc);
    HT10(1, 4 * g + 3);
    wg_barrier();
    if (++cc == nch) {
      cc = 0;
      ++it;
    }
  }
  wg_barrier();   // B_end
  if (!HDBG10(2)) {   // the last tile's store (its x loads in place)
    Tp = Tc;
    for (int u = 0; u < 4; ++u) {
      u32x4 tmp[4];
      unit_load(nt, u, tmp);
      unit_run(nt, u, tmp);
    }
  }
}

int g_ncu = 0;
int g_halo10 = -1;   // FMD_HALO10=1 enables v10 (measured slower than v9b except plain forwards)

}  // namespace

// v10 for a problem fmd_conv_halo has set up in A: returns 1 when it does not apply (v9b / older kernels then run it)
int halo10_launch(const HArgs& A, int pro, fmd_stream_t stream) {
  if (g_halo10 < 0) {
    const char* e = getenv("FMD_HALO10");
    g_halo10 = (e && *e) ? atoi(e) : 0;
  }
  const fmd_conv_desc* d = &A.d;
  if (!g_halo10 || A.splits > 1 || d->upsample || d->gout || d->out_f32 || d->accumulate) return 1;
  if (d->K % BCO || (d->resid && d->ep_x0) || A.nchunk1 + A.nchunk2 < 2 || A.nchunk1 < 1) return 1;
  if (d->ep_a && !d->ep_x0) return 1;
  if ((long long)d->Hs * d->Ws >= (1LL << 24) || (long long)d->N * d->Ho * d->Wo >= (1LL << 24)) return 1;   // __umul24
  if (d->ep_x0 && (d->ep_C0 % 8 || (d->ep_C0 < d->K && !d->ep_x1))) return 1;
  const int ntiles = d->N * A.tiles_x * A.tiles_y * A.ntc;
  if (!g_ncu) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess ||
        hipDeviceGetAttribute(&g_ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      g_ncu = 256;
    if (g_ncu <= 0) g_ncu = 256;
  }
  const int G = ntiles < g_ncu ? ntiles : g_ncu;
  const int side = d->resid ? 1 : (d->ep_x0 && d->ep_a) ? 2 : 0;
  hipStream_t st = (hipStream_t)stream;
  static const int prio = [] {   // FMD_H10_PRIO: consumer priority + 4 x producer priority (default 1: consumers 1)
    const char* e = getenv("FMD_H10_PRIO");
    return e && *e ? atoi(e) & 15 : 1;
  }();
#define H10(P, S) hipLaunchKernelGGL((conv3x3_halo10<P, S>), dim3(G), dim3(NT10), 0, st, A, ntiles, prio)
  if (pro == 2) {
    if (side == 1) H10(2, 1); else if (side == 2) H10(2, 2); else H10(2, 0);
  } else if (pro == 1) {
    if (side == 1) H10(1, 1); else if (side == 2) H10(1, 2); else H10(1, 0);
  } else {
    if (side == 1) H10(0, 1); else if (side == 2) H10(0, 2); else H10(0, 0);
  }
#undef H10
  return (int)hipGetLastError();
}

// Debug hook (not part of the public ABI): 0 routes every problem to v9b, 1 back to v10 (A/B in one process).
extern "C" int fmd_debug_halo10(int on) {
  g_halo10 = on ? 1 : 0;
  return 0;
}
