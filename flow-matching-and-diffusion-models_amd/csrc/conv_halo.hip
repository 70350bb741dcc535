// Halo-tiled 3x3 stride-1 convolution for gfx950 -- the UNet's dominant problem.
//
// Workgroup = 512 threads (8 waves) computing a 16x16-pixel x 128-output-channel
// tile; two workgroups share a CU (76 KiB of LDS each), so one workgroup's
// staging, barriers, prologue and epilogue overlap the other's MFMAs.  Per
// 32-channel chunk of the input, the (16+2)x(16+2) halo of the tile is gathered
// ONCE (GroupNorm affine + SiLU applied once per element, zero padding, optional
// nearest-x2 upsample = a 10x10 low-resolution halo, optional two-source concat)
// into LDS, and all 9 taps read their shifted 16-pixel rows from that single
// image: 9x less gather/transform work and ~7x less activation traffic than a
// per-tap implicit GEMM.  Per tap, a 128x32 weight slice (pre-tiled in HBM by
// fmd_prep_weights_batch / fmd_tile_weights_halo, so each slice is one
// contiguous 8 KiB block) is copied global -> LDS by DMA into a double-buffered
// pair of tiles; two taps per step, one barrier per step, and the next chunk's
// halo is gathered in 4 pieces behind the current chunk's MFMAs.
//
// LDS images are chunk-major ([16-byte k-chunk plane][row], plane stride 336
// rows == 0 mod 16): an MFMA fragment read is 16 consecutive rows of one plane
// per 16-lane group, so every ds_read_b128 lane group of gfx950 touches 16
// distinct 16-byte bank slots for any tap shift.  Staging lanes are mapped
// 8 consecutive positions per channel group, so the 8-lane groups of
// ds_write_b128 are conflict-free too.
//
// 3-D (3x3x3, stride 1, optionally nearest-x2): the N*D output depth slices are the images and the main
// reduction runs over (depth tap kz, 32-channel block) chunks; chunk kz stages the 18x18 halo of input slice
// z + kz - 1 (zeros past either end of a sample; slice >> 1 under nearest-x2), so all 27 taps accumulate in
// one launch with the same prologue / epilogue, and the per-sample tables are indexed by slice / D.  The
// weights are pre-tiled as a 2-D conv over 3 * C32 input channels (engine WeightCache.dtiled).
//
// Same epilogue contract as csrc/conv.hip (bias, per-sample bias, residual,
// second 1x1 GEMM over src2|src3, data-gradient SiLU' + GN-backward sums,
// channel statistics).
#include "halo_args.h"

// ablation flags of the next launches (fmd_debug_halo_flags); also read by the halo weight gradient
// (csrc/wgrad_halo.hip) in FMD_HALO_DBG builds
int g_dbg = 0;

namespace {

constexpr int TH = 16, TW = 16;           // output tile
constexpr int BCO = 128;                  // output channels per tile
constexpr int BK = FMD_HALO_BK;           // input channels per chunk (32)
constexpr int KC = BK / 8;                // 16-byte chunks per position (4)
constexpr int HALO = (TH + 2) * (TW + 2); // 324 positions
constexpr int HPAD = 336;                 // plane stride (rows): == 0 mod 16 bank slots
constexpr int HBUF = KC * HPAD * 8;       // bf16 elements per halo buffer (21 KiB)
constexpr int WBUF = KC * BCO * 8;        // bf16 elements per weight tile (8 KiB = one 16 B DMA per thread)
static_assert(2 * HBUF + 4 * WBUF >= TH * TW * BCO, "epilogue tile fits in the staging LDS");

// HArgs: csrc/halo_args.h (shared with the v9 kernel, csrc/conv_halo9.hip)

#ifdef FMD_HALO_DBG
#define HDBG(bit) (A.dbg & (bit))
#else
#define HDBG(bit) false
#endif

static unsigned long long* g_tbuf = nullptr;

// Phase timeline instrumentation (-DFMD_HALO_TIME; tools/halo_timeline.py): lane 0 of waves 0 and 4 of every
// workgroup stores s_memtime at fixed points: [0] HW_ID, [1] XCC_ID, [2] start, [24] tables loaded, [25] first
// halo loads issued, [26] first halo stored, [3] prologue barrier, [4..23] after each main-loop step barrier,
// [30] loop done, [27] epilogue tile packed, [28] epilogue barrier, [31] end.  Vector stores only; the buffer
// must be armed (fmd_debug_halo_timebuf) before any launch of an instrumented build.
#ifdef FMD_HALO_TIME
#define HTIME(slot)                                                                                    \
  do {                                                                                                 \
    if ((threadIdx.x & 255) == 0)                                                                      \
      A.tbuf[((size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 2 + (threadIdx.x >> 8)) * 32 + (slot)] = \
          __builtin_amdgcn_s_memtime();                                                                \
  } while (0)
#else
#define HTIME(slot) do {} while (0)
#endif

// staged piece h (16 bytes) of a chunk: blocks of 32 = 8 consecutive positions x KC channel groups
FMD_DEV int piece_pos(int h) { return (h >> 5) * 8 + (h & 7); }
FMD_DEV int piece_kc(int h) { return (h >> 3) & (KC - 1); }

// LDS (one __shared__ object, so hipcc's LDS-DMA wait tracking sees a single staging array):
//   [2 halo buffers][4 weight tiles][GN affine table a[C] | b[C]][epilogue bias | ep_a | ep_b of the tile]
constexpr int CMAX = 512;                              // widest GN-prologue input the affine table holds
constexpr int SM_H = 0;
constexpr int SM_W = SM_H + 2 * HBUF * 2;              // bytes
constexpr int SM_COEF = SM_W + 4 * WBUF * 2;
constexpr int SM_EPI = SM_COEF + 2 * CMAX * 4;
constexpr int SM_BYTES = SM_EPI + 3 * BCO * 4;
static_assert(SM_BYTES <= 163840 / 2, "two workgroups per CU");

// end of a pipeline step: this wave's weight DMAs (and, if keep == 0, its halo prefetch) have
// landed and its LDS stores are done; then the workgroup barrier.  Raw s_barrier: __syncthreads()
// would drain the halo prefetch that is meant to stay in flight across the barrier.
template <int KEEP>
FMD_DEV void step_barrier() {
  if constexpr (KEEP == 3) asm volatile("s_waitcnt vmcnt(3) lgkmcnt(0)" ::: "memory");
  else if constexpr (KEEP == 2) asm volatile("s_waitcnt vmcnt(2) lgkmcnt(0)" ::: "memory");
  else if constexpr (KEEP == 1) asm volatile("s_waitcnt vmcnt(1) lgkmcnt(0)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  asm volatile("" ::: "memory");
}

// Workgroup: 8 waves = 2 cout halves (64 couts) x 4 pixel-row groups (4 tile rows), 128 VGPRs, 4 waves/SIMD
constexpr int NT = 512;
constexpr int WR = 4;    // output rows per wave
constexpr int NWH = 4;   // waves per cout half

// PRO: 0 = raw input, 1 = GroupNorm affine, 2 = affine + SiLU (fused prologue, applied once per halo element)
// GOUT: also write the prologue's output G to d.gout (the tile's own pixels of every main chunk it stages)
template <bool UP, int PRO, bool GOUT = false>
__global__ __launch_bounds__(512) __attribute__((amdgpu_waves_per_eu(4, 4)))
void conv3x3_halo(const HArgs A) {
  constexpr int WDMA = WBUF / (NT * 8);                    // 16-byte weight DMAs per thread per tap
  static_assert(WDMA * NT * 8 == WBUF, "weight tile DMA split");
  constexpr int HROW = UP ? TW / 2 + 2 : TW + 2;          // halo row width (10 | 18)
  constexpr int HPOS = UP ? (TH / 2 + 2) * HROW : HALO;   // positions of a main chunk (100 | 324)
  constexpr int TOT1 = ((HPOS + 7) / 8) * 8 * KC;          // staged pieces of a main chunk
  constexpr int PC1 = ((TOT1 + 3) / 4 + 31) & ~31;         // pieces staged per step (4 staging steps per chunk)
  constexpr int LPT = (PC1 + NT - 1) / NT;                 // loads per thread per staging step (1)
  constexpr int LPRO = (TOT1 + NT - 1) / NT;               // loads per thread for the prologue's full chunk
  constexpr int SEG2 = TH * TW * KC;                       // pieces of a 1x1 chunk (1024)
  static_assert(LPT >= 1 && LPT <= 2, "staged pieces per thread and step");
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM_BYTES];
  bf16r* const lds = (bf16r*)smem;
  bf16r* const hbuf = (bf16r*)(smem + SM_H);
  bf16r* const wbuf = (bf16r*)(smem + SM_W);
  float* const coef = (float*)(smem + SM_COEF);
  float* const epi = (float*)(smem + SM_EPI);   // [3][BCO]: summed bias, ep_a, ep_b of this tile's couts
  const unsigned lds_base = (unsigned)(size_t)(__attribute__((address_space(3))) unsigned char*)smem;

  const fmd_conv_desc& d = A.d;
  const int tid = threadIdx.x, lane = tid & 63, wid = tid >> 6;
  const int wco = wid / NWH, wpx = wid % NWH;
#ifdef FMD_HALO_TIME
  HTIME(2);
  if ((tid & 255) == 0) {
    unsigned long long* tb = A.tbuf + ((size_t)(blockIdx.x + gridDim.x * blockIdx.y) * 2 + (wid >> 2)) * 32;
    tb[0] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    tb[1] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // HW_REG_XCC_ID
  }
#endif   // 2 x NWH waves: 64 couts x WR pixel rows each
  const int l16 = lane & 15, lq = lane >> 4;
  const int kc = piece_kc(tid);              // staged pieces start at multiples of 32: the channel group is fixed

  const int per_img = A.tiles_x * A.tiles_y;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int tco = b % A.ntc;
  const int tile = b / A.ntc;
  const int n = tile / per_img;
  const int tin = tile - n * per_img;
  const int smp = A.depth ? n / A.depth : n;          // sample of this image (3-D: slice n of sample smp)
  const int zz = A.depth ? n - smp * A.depth : 0;
  const int ty0 = (tin / A.tiles_x) * TH, tx0 = (tin - (tin / A.tiles_x) * A.tiles_x) * TW;
  const int co0 = tco * BCO;
  const int hy0 = UP ? (ty0 >> 1) - 1 : ty0 - 1;   // halo origin (stored-input coordinates)
  const int hx0 = UP ? (tx0 >> 1) - 1 : tx0 - 1;

  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;
  const bf16r* __restrict__ s2 = (const bf16r*)d.src2;
  const bf16r* __restrict__ s3 = (const bf16r*)d.src3;

  // the GN affine of image n for every input channel, and the epilogue's per-cout vectors
  if (PRO != 0) {
    for (int i = tid; i < 2 * A.C; i += NT)
      coef[i] = i < A.C ? d.pro_a[(size_t)smp * A.C + i] : d.pro_b[(size_t)smp * A.C + (i - A.C)];
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

  // ---- weights: one contiguous 8 KiB tile per tap, copied global -> LDS by the DMA path
  // slot = tap index over the whole reduction: 9 per 3x3 chunk, then 1 per 1x1 chunk; wtile = 0..3.
  // Wave-uniform source base (SGPRs) + this lane's fixed 16-byte offset: no per-DMA vector address math.
  static_assert(WDMA == 1, "one 16-byte weight DMA per thread and tap");
  const int T1 = A.nchunk1 * 9;
  const bf16r* const wbase1 = A.wt + (size_t)tco * T1 * WBUF;
  const bf16r* const wbase2 = A.wt2 + (size_t)tco * A.nchunk2 * WBUF;
  const unsigned wvoff = (unsigned)tid * 16;
  const unsigned wdst0 = __builtin_amdgcn_readfirstlane(lds_base + SM_W + (unsigned)(wid * 64 * 8) * 2);
  auto load_w = [&](int slot, int wtile) {
    const bf16r* src = slot < T1 ? wbase1 + (size_t)slot * WBUF : wbase2 + (size_t)(slot - T1) * WBUF;
    glds16s(src, wvoff, wdst0 + (unsigned)(wtile * WBUF * 2));
  };

  // ---- halo staging through registers (the GN/SiLU transform happens between load and LDS store)
  constexpr int LMAX = LPRO > SEG2 / NT ? (LPRO > 2 ? LPRO : 2) : (SEG2 / NT > 2 ? SEG2 / NT : 2);
  u32x4 rh[LMAX];
  int hoff[LMAX];            // LDS element offset; -1: no store; bit 30: store zeros (padding)
  const bf16r* cbase = s0;   // this thread's channel group of the chunk being staged
  int cs = 0;                // its pixel stride
  int cch = 0;               // its first channel (GN affine table index)
  bool cok = false;
  int srcsl = n;             // stored source image of the chunk being staged (3-D: depth-tap slice)
  const int HWs = d.Hs * d.Ws;
  int cimg = n * HWs;        // its first pixel

  auto setup = [&](int chunk) {
    if (chunk < A.nchunk1) {
      int cb = chunk;
      bool zok = true;
      if (A.depth) {
        const int kz = chunk / A.ncb;
        cb = chunk - kz * A.ncb;
        const int zl = zz + kz - 1;                 // logical input depth == output depth (stride 1)
        zok = zl >= 0 && zl < A.depth;
        srcsl = smp * A.dsrc + (UP ? zl >> 1 : zl);
        cimg = srcsl * HWs;
      }
      const int c = cb * BK + kc * 8;
      cok = c < A.C && zok;
      cbase = !cok ? s0 : (c < d.C0) ? s0 + c : s1 + (c - d.C0);
      cs = (c < d.C0) ? d.C0 : d.C1;
      cch = cok ? c : 0;
    } else {
      const int c = (chunk - A.nchunk1) * BK + kc * 8;
      cok = c < A.C23;
      cbase = !cok ? s2 : (c < d.C2) ? s2 + c : s3 + (c - d.C2);
      cs = (c < d.C2) ? d.C2 : d.C3;
      cch = 0;
    }
  };
  // address + LDS destination of staged piece h (main chunk: halo position; 1x1 chunk: interior pixel).
  // One load instruction whichever the source, so no branch-dependent register hazards reach the loop.
  auto piece_src = [&](int h, bool act, bool seg2, int& off) -> const bf16r* {
    const int pos = piece_pos(h);
    int pix, lpos;
    bool valid;
    if (!seg2) {
      const bool on = act && pos < HPOS;
      const int py = pos / HROW, px = pos - (pos / HROW) * HROW;   // constant divisor: mul-shift
      const int y = hy0 + py, x = hx0 + px;
      valid = on && cok && y >= 0 && y < d.Hs && x >= 0 && x < d.Ws;
      pix = (srcsl * d.Hs + y) * d.Ws + x;
      lpos = pos;
      act = on;
    } else {
      const int py = pos >> 4, px = pos & 15;
      pix = (n * d.Ho + ty0 + py) * d.Wo + tx0 + px;
      valid = act && cok;
      lpos = (py + 1) * (TW + 2) + px + 1;
    }
    off = !act ? -1 : ((kc * HPAD + lpos) * 8) | (valid ? 0 : (1 << 30));
    return cbase + (valid ? pix : 0) * cs;
  };
  auto load_main = [&](int k, int h, bool act) {
    int off;
    const bf16r* src = piece_src(h, act, false, off);
    rh[k] = *(const u32x4*)src;
    hoff[k] = off;
  };
  auto load_seg2 = [&](int k, int h, bool act) {
    int off;
    const bf16r* src = piece_src(h, act, true, off);
    rh[k] = *(const u32x4*)src;
    hoff[k] = off;
  };
  auto store = [&](int buf, int k, bool transform, int c) {
    u32x4 v = rh[k];
    if (PRO != 0 && transform && !HDBG(2)) {
      const f32x4 a0 = *(const f32x4*)(coef + c), a1 = *(const f32x4*)(coef + c + 4);
      const f32x4 b0 = *(const f32x4*)(coef + A.C + c), b1 = *(const f32x4*)(coef + A.C + c + 4);
      const float ca[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const float cb[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = bf_lo(v[e]) * ca[2 * e] + cb[2 * e];
        float hi = bf_hi(v[e]) * ca[2 * e + 1] + cb[2 * e + 1];
        if (PRO == 2) { lo = siluf_(lo); hi = siluf_(hi); }
        v[e] = pack2(lo, hi);
      }
    }
    const int o = hoff[k];
    if (o & (1 << 30)) v = u32x4{0u, 0u, 0u, 0u};
    if (o >= 0) *(u32x4*)(hbuf + buf * HBUF + (o & ~(1 << 30))) = v;
  };

  f32x4 acc[4][WR];

  // per-thread staging geometry of a main chunk, the same for every chunk of the tile: the piece of staging
  // step q (0..3) is halo position ppos0 + q * PC1 / 4 of channel group kc (PC1 % 32 == 0)
  static_assert(LPT == 1 && PC1 % 32 == 0, "one staged piece per thread and step");
  const int ppos0 = piece_pos(tid);
  int spix0, spix1, spix2, spix3;   // its pixel inside the stored image; -1 zero padding; -2 nothing to stage
  {
    int sp[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int pos = ppos0 + q * (PC1 / 4);
      const bool on = tid < PC1 && q * PC1 + tid < TOT1 && pos < HPOS;
      const int py = pos / HROW, px = pos - (pos / HROW) * HROW;
      const int y = hy0 + py, x = hx0 + px;
      sp[q] = !on ? -2 : (y >= 0 && y < d.Hs && x >= 0 && x < d.Ws) ? y * d.Ws + x : -1;
    }
    spix0 = sp[0]; spix1 = sp[1]; spix2 = sp[2]; spix3 = sp[3];
  }
  const int sl0 = (kc * HPAD + ppos0) * 8;

  auto compute = [&](int hb_i, int tap, bool seg2, int wb_i) {
    const bf16r* hb = hbuf + hb_i * HBUF;
    const bf16r* wb = wbuf + wb_i * WBUF;
    const int ky = tap / 3, kx = tap - (tap / 3) * 3;
    bf16x8 af[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) af[i] = *(const bf16x8*)(wb + (lq * BCO + wco * 64 + 16 * i + l16) * 8);
    auto bfrag = [&](int j) -> bf16x8 {
      const int py = wpx * WR + j;
      int pos;
      if (UP && !seg2) {
        const int ly = ((ty0 + py + ky - 1) >> 1) - hy0;
        const int lx = ((tx0 + l16 + kx - 1) >> 1) - hx0;
        pos = ly * HROW + lx;
      } else {
        pos = (py + ky) * (TW + 2) + l16 + kx;
      }
      return *(const bf16x8*)(hb + (lq * HPAD + pos) * 8);
    };
#pragma unroll
    for (int j = 0; j < WR; ++j) {
      const bf16x8 bv = bfrag(j);
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[i][j] = mfma16(af[i], bv, acc[i][j]);
    }
  };

  // ---- this workgroup's reduction range (split-K over 3x3 chunks; the 1x1 segment goes to the last split)
  const int split = blockIdx.y;
  const int c_lo = split * A.cps, c_hi = min(A.nchunk1, c_lo + A.cps);
  const int n_seg2 = split == A.splits - 1 ? A.nchunk2 : 0;
  const int slot_end = n_seg2 ? T1 + n_seg2 : c_hi * 9;   // one past the last weight slot of this split
  auto next_chunk = [&](int c) { return c + 1 < c_hi ? c + 1 : (c + 1 == c_hi && n_seg2 ? A.nchunk1 : -1); };

  // ---- prologue: the full halo of the first chunk (always a 3x3 chunk) + the weights of its first step
  HTIME(24);
  __syncthreads();   // affine + epilogue tables (no DMA in flight yet)
  setup(c_lo);
  load_w(c_lo * 9, 0);
  if (c_lo * 9 + 1 < slot_end) load_w(c_lo * 9 + 1, 1);
#pragma unroll
  for (int k = 0; k < LPRO; ++k) load_main(k, tid + NT * k, tid + NT * k < TOT1);
  HTIME(25);
#pragma unroll
  for (int k = 0; k < LPRO; ++k) store(c_lo & 1, k, true, cch);
  HTIME(26);
#pragma unroll
  for (int i = 0; i < 4; ++i)
#pragma unroll
    for (int j = 0; j < WR; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  step_barrier<0>();
  HTIME(3);

  // ---- 3x3 chunks: 5 steps of taps (0,1) (2,3) (4,5) (6,7) (8).  The next chunk's halo is staged in
  //      4 pieces: piece i is loaded into registers in step i (after that step's weight DMA, so the
  //      DMA's counted wait leaves it in flight across the barrier) and transformed + stored in step
  //      i+1.  Waves of the two cout halves share a SIMD pairwise: wco 0 stores before its first tap,
  //      wco 1 after it, so one wave's GroupNorm/SiLU VALU work overlaps the other's MFMAs.
  // G side output (GOUT): the tile's own pixels of a main chunk's staged (transformed) halo image, copied
  // LDS -> d.gout ((C0+C1) % 32 == 0, checked on the host).  Chunk c's image is copied in step 0 of chunk
  // c + 1 after that step's loads, so the step barrier's counted wait leaves these stores in flight (they are
  // the youngest vector-memory ops); the last chunk's image right after the loop.  Returns the stores this
  // wave issued.
  auto copy_g = [&](int gc) -> int {
    if constexpr (!GOUT) {
      return 0;
    } else {
      constexpr int IH = UP ? TH / 2 : TH, IW = UP ? TW / 2 : TW;   // the tile's own stored pixels
      constexpr int NPG = IH * IW * KC;                            // 16-byte pieces (1024 | 256)
      static_assert(NPG % NT == 0 || NPG * 2 == NT, "whole waves per copied piece row");
      int cb = gc, kzc = 1;
      if (A.depth) { kzc = gc / A.ncb; cb = gc - kzc * A.ncb; }
      // 3-D: the centre depth tap only; under nearest-x2 the even output slice of each stored slice
      if (kzc != 1 || (A.depth && UP && (zz & 1))) return 0;
      // opaque copies: the address math stays here instead of being hoisted out of the chunk loop
      int t_ = tid, ty_ = ty0, tx_ = tx0, img = A.depth ? smp * A.dsrc + (UP ? zz >> 1 : zz) : n;
      asm volatile("" : "+v"(t_), "+v"(ty_), "+v"(tx_), "+v"(img));
      const int oy = UP ? ty_ >> 1 : ty_, ox = UP ? tx_ >> 1 : tx_;
      const bf16r* hb = hbuf + (gc & 1) * HBUF;
      int nst = 0;
#pragma unroll
      for (int q = 0; q < (NPG + NT - 1) / NT; ++q) {
        if (NPG >= NT || wid < NPG / 64) {   // wave-uniform
          const int h = t_ + q * NT;
          // 4 consecutive lanes = the chunk's 64 contiguous bytes of one pixel
          const int kq = h & (KC - 1), px = (h / KC) % IW, py = h / (KC * IW);
          const int c = cb * BK + kq * 8;
          const u32x4 v = *(const u32x4*)(hb + (kq * HPAD + (py + 1) * HROW + px + 1) * 8);
          const size_t pix = ((size_t)img * d.Hs + oy + py) * d.Ws + ox + px;
          *(u32x4*)((bf16r*)d.gout + pix * A.C + c) = v;
          ++nst;
        }
      }
      return nst;
    }
  };

  int wb = 0;   // weight double-buffer of the current step (tiles 2*wb, 2*wb+1)
  int pc = 0;   // affine-table channel of the pending piece
  for (int chunk = c_lo; chunk < c_hi; ++chunk) {
    const int nx = next_chunk(chunk);
    const bool more = nx >= 0, nseg2 = nx >= A.nchunk1;
#pragma unroll 1
    for (int ps = 0; ps < 5; ++ps) {
      const int slot = chunk * 9 + 2 * ps;
      const bool two = ps < 4;
      const bool pend = more && ps > 0;    // piece ps-1 of chunk nx waits in registers
      const bool issue = more && ps < 4;   // piece ps of chunk nx is loaded this step
      auto issue_loads = [&]() {
        // weights of the next step: the next pair of this chunk, the first pair of the next chunk,
        // or the first 1x1 slot
        const int nslot = two ? slot + 2 : (nx < 0 ? slot_end : nx < A.nchunk1 ? nx * 9 : T1 + (nx - A.nchunk1));
        if (nslot < slot_end && !HDBG(8)) {
          load_w(nslot, 2 * (wb ^ 1));
          const bool ntwo = nslot < T1 && (nslot - (nslot / 9) * 9) < 8;
          if (ntwo) load_w(nslot + 1, 2 * (wb ^ 1) + 1);
        }
        // one halo load per step, always (a dummy in-bounds read when nothing is staged): the register
        // then has the same load -> consume pattern on every path, so hipcc's waits stay counted
        if (issue && ps == 0) setup(nx);
        int off;
        const bf16r* src;
        if (!nseg2) {   // main chunk: the precomputed geometry of step ps (uniform select chain)
          const int sp = ps == 0 ? spix0 : ps == 1 ? spix1 : ps == 2 ? spix2 : ps == 3 ? spix3 : -2;
          const bool act = issue && sp != -2;
          const bool valid = act && cok && sp >= 0;
          src = cbase + (valid ? cimg + sp : 0) * cs;
          off = !act ? -1 : (sl0 + ps * (PC1 / 4) * 8) | (valid ? 0 : (1 << 30));
        } else {
          src = piece_src(ps * (SEG2 / 4) + tid, issue && tid < SEG2 / 4, true, off);
        }
        if (HDBG(1)) {
          rh[0] = u32x4{0u, 0u, 0u, 0u};
        } else {
          rh[0] = *(const u32x4*)src;
        }
        hoff[0] = off;
      };
      auto consume = [&]() {   // the previous step's halo loads are consumed here, on every path
#pragma unroll
        for (int k = 0; k < LPT; ++k) asm volatile("" ::"v"(rh[k]));
      };
      auto store_pending = [&]() {
        if (pend) {
#pragma unroll
          for (int k = 0; k < LPT; ++k) store(nx & 1, k, !nseg2, pc);
        }
      };
      // Waves w and w+4 share a SIMD: the wco 0 wave stages (GN/SiLU VALU work) before its first tap,
      // the wco 1 wave after it, so one wave's transform overlaps the other's MFMAs.
      int gst = 0;   // G stores issued by this wave this step (younger than its loads)
      if (wco == 0) {
        consume();
        store_pending();
        issue_loads();
        if (GOUT && ps == 0 && chunk > c_lo) gst = copy_g(chunk - 1);
        compute(chunk & 1, 2 * ps, false, 2 * wb);
      } else {
        compute(chunk & 1, 2 * ps, false, 2 * wb);
        consume();
        store_pending();
        issue_loads();
        if (GOUT && ps == 0 && chunk > c_lo) gst = copy_g(chunk - 1);
      }
      pc = cch;
      if (two) compute(chunk & 1, 2 * ps + 1, false, 2 * wb + 1);
      if (GOUT && gst == 2) step_barrier<LPT + 2>();
      else if (GOUT && gst == 1) step_barrier<LPT + 1>();
      else step_barrier<LPT>();
      HTIME(4 + (chunk - c_lo) * 5 + ps);
      wb ^= 1;
    }
  }
#pragma unroll
  for (int k = 0; k < LPT; ++k) asm volatile("" ::"v"(rh[k]));
  if (GOUT && c_hi > c_lo) {   // the last main chunk's image, before the 1x1 staging / epilogue reuse its LDS
    copy_g(c_hi - 1);
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
  }
  // ---- 1x1 chunks (ResBlock skip conv over src2|src3): one step each, next chunk staged whole
  for (int chunk = A.nchunk1; chunk < A.nchunk1 + n_seg2; ++chunk) {
    const int nx = chunk + 1;
    const bool more = nx < A.nchunk1 + n_seg2;
    const int slot = T1 + (chunk - A.nchunk1);
    if (slot + 1 < slot_end) load_w(slot + 1, 2 * (wb ^ 1));
    if (more) {
      setup(nx);
#pragma unroll
      for (int k = 0; k < SEG2 / NT; ++k) load_seg2(k, tid + NT * k, true);
    }
    compute(chunk & 1, 4, true, 2 * wb);
    if (more) {
#pragma unroll
      for (int k = 0; k < SEG2 / NT; ++k) store(nx & 1, k, false, 0);
    }
    step_barrier<0>();
    wb ^= 1;
  }

  HTIME(30);
  if (HDBG(4)) return;
  // ------------------------------------------------------------ epilogue
  const int K = d.K;
  const int Ho = d.Ho, Wo = d.Wo;
  if (A.splits > 1) {   // fp32 partial sums of this split; splitk_reduce applies the epilogue
    float* ws = d.ws + (size_t)split * d.N * Ho * Wo * K;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + wco * 64 + 16 * i + 4 * lq;
      if (co >= K) continue;
#pragma unroll
      for (int j = 0; j < WR; ++j) {
        const size_t p = ((size_t)n * Ho + ty0 + wpx * WR + j) * Wo + tx0 + l16;
        if (co + 3 < K) {
          *(f32x4*)(ws + p * K + co) = acc[i][j];
        } else {
          for (int r = 0; r < 4; ++r)
            if (co + r < K) ws[p * K + co + r] = acc[i][j][r];
        }
      }
    }
    return;
  }
  const bool stats = d.stats != nullptr;
  const bool dep = d.ep_a != nullptr;
  const bool hasx = d.ep_x0 != nullptr;
  // per-channel sums of this lane's 4 pixels, reduced over the wave's 16 pixel lanes per cout block:
  // slab row = 64 pixels (4 tile rows x 16) of one image; any bijection works for GN
  auto flush_stats = [&](int i, int j0, const float* a4, const float* q4) {
    const int srow = tile * 4 + (wpx * WR + j0) / 4;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const float a = row16_sum_to_last(a4[r]), q = row16_sum_to_last(q4[r]);
      const int co = co0 + wco * 64 + 16 * i + 4 * lq + r;
      if (l16 == 15 && co < K) {
        float* sp = d.stats + ((size_t)srow * K + co) * 2;
        sp[0] = a;
        sp[1] = q;
      }
    }
  };

  if (co0 + BCO <= K && !d.out_f32 && !d.accumulate && !(d.resid && hasx)) {
    // Fast path: the 256-pixel x 128-channel tile goes through LDS ([pixel][16-byte chunk ^ (pixel & 15)],
    // conflict-free for the lanes' 8-byte reads), so every global access is a coalesced 16-byte one.
    bf16r* tileb = lds;   // 64 KiB inside the (now idle) halo + weight buffers
    const bool side = d.resid != nullptr || hasx;
    if (side) {
      // the whole 64 KiB side tile in flight at once (the main loop's fragments are dead here)
      constexpr int SK = TH * TW * BCO / 8 / NT;   // 16-byte pieces per thread (8 | 16)
      u32x4 sv[SK];
#pragma unroll
      for (int k = 0; k < SK; ++k) {
        const int q = tid + NT * k, pi = q >> 4, c16 = q & 15;
        const int p = (n * Ho + ty0 + (pi >> 4)) * Wo + tx0 + (pi & 15);
        const int c = co0 + c16 * 8;
        const bf16r* src = d.resid ? (const bf16r*)d.resid + (size_t)p * K + c
                           : (c < d.ep_C0) ? (const bf16r*)d.ep_x0 + (size_t)p * d.ep_C0 + c
                                           : (const bf16r*)d.ep_x1 + (size_t)p * (K - d.ep_C0) + (c - d.ep_C0);
        sv[k] = HDBG(64) ? u32x4{0u, 0u, 0u, 0u} : *(const u32x4*)src;
      }
#pragma unroll
      for (int k = 0; k < SK; ++k) {
        const int q = tid + NT * k, pi = q >> 4, c16 = q & 15;
        *(u32x4*)(tileb + pi * BCO + ((c16 ^ (pi & 15)) * 8)) = sv[k];
      }
      __syncthreads();
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int cl = wco * 64 + 16 * i + 4 * lq;   // channel within the tile (multiple of 4)
      const int co = co0 + cl;
      const f32x4 bias = *(const f32x4*)(epi + cl);
      const f32x4 ea = *(const f32x4*)(epi + BCO + cl), eb = *(const f32x4*)(epi + 2 * BCO + cl);
      float st1[4] = {0.f, 0.f, 0.f, 0.f}, st2[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
      for (int j = 0; j < WR; ++j) {
        const int pi = (wpx * WR + j) * 16 + l16;
        bf16r* tp8 = tileb + pi * BCO + (((cl >> 3) ^ (pi & 15)) * 8) + (cl & 7);
        float v[4], xv[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[r];
        if (side) {
          const u32x2 sr = *(const u32x2*)tp8;
          const float f[4] = {bf_lo(sr[0]), bf_hi(sr[0]), bf_lo(sr[1]), bf_hi(sr[1])};
          if (d.resid) {
#pragma unroll
            for (int r = 0; r < 4; ++r) v[r] += f[r];
          } else {
#pragma unroll
            for (int r = 0; r < 4; ++r) {
              xv[r] = f[r];
              if (dep && !HDBG(16)) v[r] *= silu_grad(ea[r] * f[r] + eb[r]);
            }
          }
        }
        u32x2 o;
        o[0] = pack2(v[0], v[1]);
        o[1] = pack2(v[2], v[3]);
        *(u32x2*)tp8 = o;
        if (stats && !HDBG(32)) {
          const float w[4] = {bf_lo(o[0]), bf_hi(o[0]), bf_lo(o[1]), bf_hi(o[1])};
#pragma unroll
          for (int r = 0; r < 4; ++r) {
            st1[r] += w[r];
            st2[r] += hasx ? w[r] * xv[r] : w[r] * w[r];
          }
        }
        if (stats && (j & 3) == 3) {   // one slab row per 4 tile rows
          flush_stats(i, j - 3, st1, st2);
#pragma unroll
          for (int r = 0; r < 4; ++r) { st1[r] = 0.f; st2[r] = 0.f; }
        }
      }
    }
    HTIME(27);
    __syncthreads();
    HTIME(28);
#pragma unroll
    for (int k = 0; k < TH * TW * BCO / 8 / NT; ++k) {
      const int q = tid + NT * k, pi = q >> 4, c16 = q & 15;
      const int p = (n * Ho + ty0 + (pi >> 4)) * Wo + tx0 + (pi & 15);
      *(u32x4*)((bf16r*)d.out + (size_t)p * K + co0 + c16 * 8) =
          *(const u32x4*)(tileb + pi * BCO + ((c16 ^ (pi & 15)) * 8));
    }
  } else {
  #pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + wco * 64 + 16 * i + 4 * lq;
      if (co >= K) continue;
      const bool full = co + 3 < K;
      float bias[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < 4; ++r) {
        if (co + r < K) {
          if (d.bias) bias[r] += d.bias[co + r];
          if (d.bias2) bias[r] += d.bias2[co + r];
          if (d.bias_nc) bias[r] += d.bias_nc[(size_t)smp * K + co + r];
        }
      }
      float st1[4] = {0.f, 0.f, 0.f, 0.f}, st2[4] = {0.f, 0.f, 0.f, 0.f};
  #pragma unroll
      for (int j = 0; j < WR; ++j) {
        const int y = ty0 + wpx * WR + j, x = tx0 + l16;
        const size_t p = ((size_t)n * Ho + y) * Wo + x;
        float v[4];
  #pragma unroll
        for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[r];
        if (d.resid) {
          const bf16r* rp = (const bf16r*)d.resid + p * K + co;
          if (full) {
            const u32x2 rr = *(const u32x2*)rp;
            v[0] += bf_lo(rr[0]); v[1] += bf_hi(rr[0]); v[2] += bf_lo(rr[1]); v[3] += bf_hi(rr[1]);
          } else {
            for (int r = 0; r < 4; ++r)
              if (co + r < K) v[r] += bf2f(rp[r]);
          }
        }
        float xv[4] = {0.f, 0.f, 0.f, 0.f};
        if (hasx) {
          const int C0e = d.ep_C0;
          for (int r = 0; r < 4; ++r) {
            const int c = co + r;
            if (c >= K) continue;
            const bf16r* xp = (c < C0e) ? (const bf16r*)d.ep_x0 + p * C0e + c
                                        : (const bf16r*)d.ep_x1 + p * (K - C0e) + (c - C0e);
            xv[r] = bf2f(*xp);
            if (dep) v[r] *= silu_grad(d.ep_a[(size_t)smp * K + c] * xv[r] + d.ep_b[(size_t)smp * K + c]);
          }
        }
        if (d.out_f32) {
          float* op = (float*)d.out + p * K + co;
          for (int r = 0; r < 4; ++r)
            if (co + r < K) op[r] = d.accumulate ? op[r] + v[r] : v[r];
        } else {
          bf16r* op = (bf16r*)d.out + p * K + co;
          if (full) {
            if (d.accumulate) {
              const u32x2 o = *(const u32x2*)op;
              v[0] += bf_lo(o[0]); v[1] += bf_hi(o[0]); v[2] += bf_lo(o[1]); v[3] += bf_hi(o[1]);
            }
            u32x2 o;
            o[0] = pack2(v[0], v[1]);
            o[1] = pack2(v[2], v[3]);
            *(u32x2*)op = o;
            v[0] = bf_lo(o[0]); v[1] = bf_hi(o[0]); v[2] = bf_lo(o[1]); v[3] = bf_hi(o[1]);
          } else {
            for (int r = 0; r < 4; ++r)
              if (co + r < K) {
                const float w = d.accumulate ? bf2f(op[r]) + v[r] : v[r];
                op[r] = (bf16r)f2bf(w);
                v[r] = bf2f(op[r]);
              }
          }
        }
        if (stats) {
  #pragma unroll
          for (int r = 0; r < 4; ++r) {
            st1[r] += v[r];
            st2[r] += hasx ? v[r] * xv[r] : v[r] * v[r];
          }
          if ((j & 3) == 3) {
            flush_stats(i, j - 3, st1, st2);
  #pragma unroll
            for (int r = 0; r < 4; ++r) { st1[r] = 0.f; st2[r] = 0.f; }
          }
        }
      }
    }
  }
  HTIME(31);
}

// [K][T][C] kernel-layout bf16 weights -> halo tiles [ntc][nchunk][T][KC][BCO][8] (zero padded)
__global__ void tile_weights_kernel(const bf16r* __restrict__ w, int K, int T, int C, int ntc, int nchunk,
                                    bf16r* __restrict__ out) {
  const long long total = (long long)ntc * nchunk * T * KC * BCO * 8;
  for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
       i += (long long)gridDim.x * blockDim.x) {
    const int e = (int)(i & 7);
    long long r = i >> 3;
    const int co = (int)(r % BCO); r /= BCO;
    const int kc = (int)(r % KC); r /= KC;
    const int tap = (int)(r % T); r /= T;
    const int chunk = (int)(r % nchunk);
    const int tc = (int)(r / nchunk);
    const int k = tc * BCO + co, c = chunk * BK + kc * 8 + e;
    out[i] = (k < K && c < C) ? w[((size_t)k * T + tap) * C + c] : (bf16r)0;
  }
}

}  // namespace

// Called by fmd_conv when the problem qualifies (3x3, stride 1, pad 1, forward gather,
// output tile 16x16 inside one image, >= 128 tiles).  Returns 1 if not applicable.
// fewest workgroups (tiles x splits) the halo conv takes; smaller grids go to the implicit GEMM
// (32: config D's latent sampler 81.7 / 81.4 -> 77.4 / 77.3 ms per 50 steps vs 128, interleaved A/B; the config B
// train step unchanged within noise)
static int g_halo_min_wg = 32;

extern "C" int fmd_halo_set_min_workgroups(int32_t n) {
  if (n < 1) return -1;
  g_halo_min_wg = n;
  return 0;
}

extern "C" int fmd_conv_halo(const fmd_conv_desc* d, fmd_stream_t stream) {
  if (d->ks != 3 || d->stride != 1 || d->pad != 1 || d->transposed) return 1;
  const bool d3 = d->Do > 0 || d->Ds > 0;
  if (d3 && d->Do != (d->upsample ? 2 * d->Ds : d->Ds)) return 1;   // 3-D: stride-1 3x3x3 (nearest-x2)
  const int Nn = d3 ? d->N * d->Do : d->N;                // images (3-D: depth slices)
  if (d->splits > 1 && (!d->ws || (d->stats && !d->tickets))) return 1;   // ticketed splits: statistics in the epilogue
  if (d->Ho % TH || d->Wo % TW) return 1;
  if (d->upsample ? (d->Ho != 2 * d->Hs || d->Wo != 2 * d->Ws) : (d->Ho != d->Hs || d->Wo != d->Ws)) return 1;
  if (!d->wgt_tiled || (d->src2 && !d->wgt2_tiled)) return 1;
  if ((d->pro_a || d->fold_st0) && d->C0 + d->C1 > CMAX) return 1;   // the GN affine table holds CMAX channels
  if (d->fold_st0 && (d3 || d->gout || d->pro_a || d->fold_G < 1 || (d->C0 + d->C1) % d->fold_G || d->fold_rows0 < 1 ||
                      (d->Hs * d->Ws) % d->fold_rows0 ||
                      (d->C1 && (!d->fold_st1 || d->fold_rows1 < 1 || (d->Hs * d->Ws) % d->fold_rows1))))
    return 1;   // the in-kernel fold: 2-D, whole slab rows, one source of statistics per input
  if (d->gout && (d->C0 + d->C1) % BK) return 1;     // G side output: whole 32-channel chunks
  if ((long long)Nn * d->Hs * d->Ws * (d->C0 > d->C1 ? d->C0 : d->C1) >= (1LL << 31) ||
      (long long)Nn * d->Ho * d->Wo * (d->C2 > d->C3 ? d->C2 : d->C3) >= (1LL << 31)) return 1;   // 32-bit offsets
  HArgs A;
  A.d = *d;
  A.C = d->C0 + d->C1;
  A.C23 = d->src2 ? d->C2 + d->C3 : 0;
  A.tiles_x = d->Wo / TW;
  A.tiles_y = d->Ho / TH;
  A.ntc = (d->K + BCO - 1) / BCO;
  A.depth = d3 ? d->Do : 0;
  A.dsrc = d3 ? d->Ds : 0;
  A.ncb = (A.C + BK - 1) / BK;
  A.nchunk1 = d3 ? 3 * A.ncb : A.ncb;   // 3-D: weights pre-tiled as a 3*ncb*32-channel 2-D conv (kz-major)
  A.d.N = Nn;
  A.nchunk2 = d->src2 ? (A.C23 + BK - 1) / BK : 0;
  A.nsteps_slots = A.nchunk1 * 9 + A.nchunk2;
  A.splits = d->splits > 1 ? d->splits : 1;
  A.cps = (A.nchunk1 + A.splits - 1) / A.splits;
  if (A.splits > 1 && (A.splits - 1) * A.cps >= A.nchunk1) return 1;   // every split owns >= 1 chunk
  A.wt = (const bf16r*)d->wgt_tiled;
  A.wt2 = (const bf16r*)d->wgt2_tiled;
  A.fold_E0 = d->fold_st0 ? d->Hs * d->Ws / d->fold_rows0 : 0;
  A.fold_E1 = d->fold_st0 && d->C1 ? d->Hs * d->Ws / d->fold_rows1 : 0;
  A.fold_inv = d->fold_st0 ? 1.0 / ((double)(A.C / d->fold_G) * d->Hs * d->Ws) : 0.0;
  A.dbg = g_dbg;
  A.tbuf = g_tbuf;
  const int nwg = Nn * A.tiles_x * A.tiles_y * A.ntc;
  if (nwg * A.splits < g_halo_min_wg) return 1;   // too few workgroups to fill the chip: the implicit GEMM wins
  const int pro = d->pro_a || d->fold_st0 ? (d->pro_silu ? 2 : 1) : 0;
  {   // the v9b kernel (csrc/conv_halo9.hip) takes every problem it supports
    const int rc9 = halo9_launch(A, pro, stream);
    if (rc9 != 1 || d->fold_st0 || (d->tickets && A.splits > 1)) return rc9;   // the fold and the in-launch combine exist only in v9b
  }
  hipStream_t st = (hipStream_t)stream;
  const dim3 g(nwg, A.splits);
  const dim3 blk(NT);
  if (d->gout) {   // prologue side output (fmd_conv checked pro_a)
    if (d->upsample) {
      if (pro == 2) hipLaunchKernelGGL((conv3x3_halo<true, 2, true>), g, blk, 0, st, A);
      else hipLaunchKernelGGL((conv3x3_halo<true, 1, true>), g, blk, 0, st, A);
    } else {
      if (pro == 2) hipLaunchKernelGGL((conv3x3_halo<false, 2, true>), g, blk, 0, st, A);
      else hipLaunchKernelGGL((conv3x3_halo<false, 1, true>), g, blk, 0, st, A);
    }
    return (int)hipGetLastError();
  }
  if (d->upsample) {
    if (pro == 2) hipLaunchKernelGGL((conv3x3_halo<true, 2>), g, blk, 0, st, A);
    else if (pro == 1) hipLaunchKernelGGL((conv3x3_halo<true, 1>), g, blk, 0, st, A);
    else hipLaunchKernelGGL((conv3x3_halo<true, 0>), g, blk, 0, st, A);
  } else {
    if (pro == 2) hipLaunchKernelGGL((conv3x3_halo<false, 2>), g, blk, 0, st, A);
    else if (pro == 1) hipLaunchKernelGGL((conv3x3_halo<false, 1>), g, blk, 0, st, A);
    else hipLaunchKernelGGL((conv3x3_halo<false, 0>), g, blk, 0, st, A);
  }
  return (int)hipGetLastError();
}

// Debug hook (not part of the public ABI): ablation flags of the next launches (see HArgs::dbg).
extern "C" int fmd_debug_halo_flags(int flags) {
  g_dbg = flags;
  return 0;
}

// Debug hook (not part of the public ABI): phase-timestamp buffer of an instrumented build (see HTIME).
extern "C" int fmd_debug_halo_timebuf(void* buf) {
  g_tbuf = (unsigned long long*)buf;
  return 0;
}

extern "C" int64_t fmd_halo_tiled_size(int32_t K, int32_t T, int32_t C) {
  return (int64_t)((K + BCO - 1) / BCO) * ((C + BK - 1) / BK) * T * KC * BCO * 8;
}

extern "C" int fmd_tile_weights_halo(const void* w, int32_t K, int32_t T, int32_t C, void* out,
                                     fmd_stream_t stream) {
  const int ntc = (K + BCO - 1) / BCO, nchunk = (C + BK - 1) / BK;
  const long long total = (long long)ntc * nchunk * T * KC * BCO * 8;
  long long blocks = (total + 255) / 256;
  if (blocks > 16384) blocks = 16384;
  hipLaunchKernelGGL(tile_weights_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (const bf16r*)w, K, T,
                     C, ntc, nchunk, (bf16r*)out);
  return (int)hipGetLastError();
}
