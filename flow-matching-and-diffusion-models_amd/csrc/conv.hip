// Implicit-GEMM convolution for gfx950 (forward and data-gradient modes).
//
// GEMM view: D[cout][pixel] = sum_{tap, cin} W[cout][tap][cin] * G[pixel][tap][cin]
// where G is the im2col gather of the (virtually concatenated, optionally
// nearest-x2-upsampled, GroupNorm-affine+SiLU-transformed) NHWC bf16 input.
// MFMA A operand = weight tile (cout rows), B operand = gathered pixel tile,
// so each lane ends with 4 consecutive output channels of one pixel (8-byte
// bf16 stores).  Tiles are staged through LDS with a 16-byte-chunk XOR swizzle
// (conflict-free ds_read_b128), double buffered with register prefetch.
//
// Replaces (reference): ConvND/nn.Conv2d (src/nn/ops/convolution.py:8-54),
// GroupNorm+SiLU(+scale/shift) feeding a conv (src/nn/blocks/residual.py:95-117),
// F.interpolate nearest x2 + conv (src/nn/ops/upsampling.py:27-29), stride-2
// DownsampleND (upsampling.py:49-56), torch.cat([h, skip]) (src/models/unet/unet.py:322),
// the 1x1 skip conv + residual add (residual.py:77-82,120), and their autograd
// data gradients (transposed gather).
#include <cstdlib>
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

struct KArgs {
  fmd_conv_desc d;
  fmd_gn_apply_desc g;   // GNA kernels: GroupNorm-backward apply epilogue (fmd_conv_gn_apply)
  int M;          // N*Ho*Wo
  int T;          // ks*ks taps
  int C;          // C0 + C1
  int nk1;        // K-iterations of the main segment: ceil(C/BK)*T
  int nk;         // total K-iterations (main + 1x1 segment)
  int per_split;  // K-iterations per split
  int ntp, ntc;   // pixel tiles, cout tiles
  int stats_rows; // pixels per stats slab row (64) or 0
  int par;        // stride-2 transposed 3x3(x3): one launch z-slice per output parity class (sub-pixel
                  // decomposition: only the 1/2/2/4 taps that hit a class are iterated, not all 9; in 3-D
                  // 8 classes of 1..8 of the 27 taps)
  int Mfull;      // N*Ho*Wo (== M unless par)
  int pack;       // 1: the input has exactly 8 (padded) channels -- one 16-byte chunk per tap -- and a K-iteration
                  // covers BK/8 consecutive TAPS (chunk j = tap kk*BK/8 + j, channels 0..7) instead of BK
                  // channels of one tap: the UNet's input conv and the 1-channel head's data gradient (K = 9
                  // or 27 taps x 8) run in ceil(T/(BK/8)) K-iterations, not T (7/8 of each was zero padding)
};

template <int BCO, int BPX, int WM, int WN, int BK, bool GNA = false>
__global__ __launch_bounds__(256, 2) void conv_igemm(const KArgs A) {
  constexpr int NT = 256;
  constexpr int CH = BK / 8;                  // 16-byte chunks per LDS row
  constexpr int RPP = NT / CH;                // rows covered per load pass
  constexpr int AW = (BCO + RPP - 1) / RPP;   // weight chunks per thread
  constexpr int AX = BPX / RPP;               // pixel chunks per thread
  constexpr int TM = BCO / (WM * 16);
  constexpr int TN = BPX / (WN * 16);
  constexpr int KS = BK / 32;
  static_assert(WM * WN == 4, "4 waves");
  static_assert(BPX % RPP == 0, "pixel tile");
  __shared__ __attribute__((aligned(16))) bf16r lds[2 * (BCO + BPX) * BK];

  const fmd_conv_desc& d = A.d;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wid = tid >> 6;
  const int wm = wid / WN, wn = wid % WN;

  const int nwg = A.ntp * A.ntc;
  const int b = xcd_remap(blockIdx.x, nwg);
  const int tco = b % A.ntc, tpx = b / A.ntc;
  const int co0 = tco * BCO, px0 = tpx * BPX;
  const int split = blockIdx.y;
  // parity class (par): output pixels (2qz + cz, 2qy + cy, 2qx + cx); taps ky in {1} (cy = 0) or {0, 2}
  // (cy = 1), likewise kx, kz (cz = 0 in 2-D)
  const bool d3 = d.Do > 0;
  const int cz = A.par && d3 ? (int)(blockIdx.z >> 2) : 0;
  const int cy = A.par ? (int)((blockIdx.z >> 1) & 1) : 0, cx = A.par ? (int)(blockIdx.z & 1) : 0;
  const int nkx = cx ? 2 : 1, nky = cy ? 2 : 1;
  const int Tc = A.par ? (cz ? 2 : 1) * nky * nkx : A.T;
  const int nk1 = A.par ? ((A.C + BK - 1) / BK) * Tc : A.nk1;
  const int nkt = A.par ? nk1 : A.nk;
  const int per_split = A.par ? (nkt + (int)gridDim.y - 1) / (int)gridDim.y : A.per_split;
  const int kk0 = split * per_split;
  const int kk1 = min(nkt, kk0 + per_split);
  const int Wq = A.par ? d.Wo >> 1 : d.Wo;
  const int Dz = d.Do > 0 ? d.Do : 1;                       // output depth (3-D problems), 1 in 2-D
  const int HWq = A.par ? (d3 ? Dz >> 1 : 1) * (d.Ho >> 1) * Wq : Dz * d.Ho * d.Wo;   // pixels per image
  const int HWp = A.par ? (d.Ho >> 1) * Wq : d.Ho * d.Wo;   // pixels per output depth slice
  // pixel index of the layout (output tensor / split-K slab) for tile pixel p
  auto pmap = [&](int p) -> int {
    if (!A.par) return p;
    const int n = p / HWq, r0 = p - n * HWq, qz = r0 / HWp, rem = r0 - qz * HWp, qy = rem / Wq, qx = rem - qy * Wq;
    return ((n * Dz + (d3 ? 2 * qz + cz : 0)) * d.Ho + 2 * qy + cy) * d.Wo + 2 * qx + cx;
  };

  const int HWo = Dz * d.Ho * d.Wo;
  const int cch = tid % CH;      // this thread's 16B chunk within a BK slice
  const int rbase = tid / CH;

  // per-thread pixel rows
  int pn[AX], poz[AX], poy[AX], pox[AX];
#pragma unroll
  for (int j = 0; j < AX; ++j) {
    const int p = px0 + rbase + j * RPP;
    if (p < A.M) {
      const int n = p / HWq;
      int rem = p - n * HWq;
      pn[j] = n;
      poz[j] = rem / HWp;
      rem -= poz[j] * HWp;
      poy[j] = rem / Wq;
      pox[j] = rem - poy[j] * Wq;
      if (A.par) { poz[j] = d3 ? 2 * poz[j] + cz : 0; poy[j] = 2 * poy[j] + cy; pox[j] = 2 * pox[j] + cx; }
    } else {
      pn[j] = -1; poz[j] = 0; poy[j] = 0; pox[j] = 0;
    }
  }
  const int Dsz = d.Ds > 0 ? d.Ds : 1;   // stored input depth

  const bf16r* __restrict__ s0 = (const bf16r*)d.src0;
  const bf16r* __restrict__ s1 = (const bf16r*)d.src1;
  const bf16r* __restrict__ s2 = (const bf16r*)d.src2;
  const bf16r* __restrict__ s3 = (const bf16r*)d.src3;
  const int C23 = d.C2 + d.C3;
  const bf16r* __restrict__ w1 = (const bf16r*)d.wgt;
  const bf16r* __restrict__ w2 = (const bf16r*)d.wgt2;
  const bool pro = d.pro_a != nullptr;

  u32x4 rw[AW], rx[AX];
  bool vx[AX];
  int cur_c = 0, cur_seg = 0;

  auto load = [&](int kk) {
    int c, tap = 0, seg;
    if (kk < nk1 && A.pack) {
      tap = kk * CH + cch;   // per-thread tap; >= T past the end (zeros)
      c = 0;
      seg = 0;
    } else if (kk < nk1) {
      const int cb = kk / Tc;
      tap = kk - cb * Tc;
      if (A.par) {   // class-local tap -> 3x3(x3) tap
        const int iz = tap / (nky * nkx), r2 = tap - iz * (nky * nkx);
        const int iy = r2 / nkx, ix = r2 - (r2 / nkx) * nkx;
        tap = (cy ? 2 * iy : 1) * 3 + (cx ? 2 * ix : 1) + (d3 ? (cz ? 2 * iz : 1) * 9 : 0);
      }
      c = cb * BK + cch * 8;
      seg = 0;
    } else {
      c = (kk - nk1) * BK + cch * 8;
      seg = 1;
    }
    cur_c = c;
    cur_seg = seg;
    const int kk2 = d.ks * d.ks;
    const int kz = tap / kk2, t2 = tap - kz * kk2;   // kz = 0 in 2-D (T = ks*ks)
    const int ky = t2 / d.ks, kx = t2 - (t2 / d.ks) * d.ks;
    // weights
#pragma unroll
    for (int j = 0; j < AW; ++j) {
      const int r = rbase + j * RPP;
      const int co = co0 + r;
      u32x4 v = {0u, 0u, 0u, 0u};
      if (r < BCO && co < d.K) {
        if (seg == 0) {
          if (c < A.C && tap < A.T) v = *(const u32x4*)(w1 + ((size_t)co * A.T + tap) * A.C + c);
        } else {
          if (c < C23) v = *(const u32x4*)(w2 + (size_t)co * C23 + c);
        }
      }
      rw[j] = v;
    }
    // activations (gather)
#pragma unroll
    for (int j = 0; j < AX; ++j) {
      const int n = pn[j];
      bool ok = n >= 0;
      const bf16r* ptr = nullptr;
      if (seg == 0) {
        int sz = 0, sy, sx;
        if (!d.transposed) {
          const int iz = d3 ? poz[j] * d.stride + kz - d.pad : 0;
          const int iy = poy[j] * d.stride + ky - d.pad;
          const int ix = pox[j] * d.stride + kx - d.pad;
          if (d.upsample) {
            ok = ok && iy >= 0 && iy < 2 * d.Hs && ix >= 0 && ix < 2 * d.Ws && iz >= 0 && iz < 2 * Dsz;
            sz = iz >> 1; sy = iy >> 1; sx = ix >> 1;
          } else {
            ok = ok && iy >= 0 && iy < d.Hs && ix >= 0 && ix < d.Ws && iz >= 0 && iz < Dsz;
            sz = iz; sy = iy; sx = ix;
          }
        } else {
          const int nz = d3 ? poz[j] + d.pad - kz : 0;
          const int ny = poy[j] + d.pad - ky;
          const int nx = pox[j] + d.pad - kx;
          ok = ok && ny >= 0 && nx >= 0 && nz >= 0;
          if (d.stride == 2) {
            ok = ok && !(ny & 1) && !(nx & 1) && !(nz & 1);
            sz = nz >> 1; sy = ny >> 1; sx = nx >> 1;
          } else {
            sz = nz; sy = ny; sx = nx;
          }
          ok = ok && sy < d.Hs && sx < d.Ws && sz < Dsz;
        }
        ok = ok && c < A.C && tap < A.T;
        if (ok) {
          const size_t pix = (((size_t)n * Dsz + sz) * d.Hs + sy) * d.Ws + sx;
          ptr = (c < d.C0) ? s0 + pix * d.C0 + c : s1 + pix * d.C1 + (c - d.C0);
        }
      } else {
        ok = ok && c < C23;
        if (ok) {
          const size_t pix = (size_t)(px0 + rbase + j * RPP);
          ptr = (c < d.C2) ? s2 + pix * d.C2 + c : s3 + pix * d.C3 + (c - d.C2);
        }
      }
      vx[j] = ok;
      rx[j] = ok ? *(const u32x4*)ptr : u32x4{0u, 0u, 0u, 0u};
    }
  };

  auto transform = [&]() {
    if (!pro || cur_seg != 0) return;
    const int c = cur_c;
#pragma unroll
    for (int j = 0; j < AX; ++j) {
      if (!vx[j]) continue;
      const float* pa = d.pro_a + (size_t)pn[j] * A.C + c;
      const float* pb = d.pro_b + (size_t)pn[j] * A.C + c;
      const f32x4 a0 = *(const f32x4*)pa, a1 = *(const f32x4*)(pa + 4);
      const f32x4 b0 = *(const f32x4*)pb, b1 = *(const f32x4*)(pb + 4);
      const float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
      const float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
      u32x4 v = rx[j];
      u32x4 o;
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        float lo = bf_lo(v[e]) * av[2 * e] + bv[2 * e];
        float hi = bf_hi(v[e]) * av[2 * e + 1] + bv[2 * e + 1];
        if (d.pro_silu) { lo = siluf_(lo); hi = siluf_(hi); }
        o[e] = pack2(lo, hi);
      }
      rx[j] = o;
    }
  };

  auto store = [&](int buf) {
    bf16r* la = lds + buf * (BCO + BPX) * BK;
    bf16r* lx = la + BCO * BK;
#pragma unroll
    for (int j = 0; j < AW; ++j) {
      const int r = rbase + j * RPP;
      if (r < BCO) *(u32x4*)(la + r * BK + 8 * (cch ^ (r & (CH - 1)))) = rw[j];
    }
#pragma unroll
    for (int j = 0; j < AX; ++j) {
      const int r = rbase + j * RPP;
      *(u32x4*)(lx + r * BK + 8 * (cch ^ (r & (CH - 1)))) = rx[j];
    }
  };

  f32x4 acc[TM][TN];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TN; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int l16 = lane & 15, lq = lane >> 4;
  auto compute = [&](int buf) {
    const bf16r* la = lds + buf * (BCO + BPX) * BK;
    const bf16r* lx = la + BCO * BK;
#pragma unroll
    for (int ks = 0; ks < KS; ++ks) {
      const int kc = 4 * ks + lq;
      bf16x8 af[TM], bfr[TN];
#pragma unroll
      for (int i = 0; i < TM; ++i) {
        const int r = wm * (BCO / WM) + 16 * i + l16;
        af[i] = *(const bf16x8*)(la + r * BK + 8 * (kc ^ (r & (CH - 1))));
      }
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int r = wn * (BPX / WN) + 16 * j + l16;
        bfr[j] = *(const bf16x8*)(lx + r * BK + 8 * (kc ^ (r & (CH - 1))));
      }
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TN; ++j) acc[i][j] = mfma16(af[i], bfr[j], acc[i][j]);
    }
  };

  if (kk0 < kk1) {
    load(kk0);
    transform();
    store(0);
    __syncthreads();
    for (int kk = kk0; kk < kk1; ++kk) {
      const int buf = (kk - kk0) & 1;
      const bool nxt = kk + 1 < kk1;
      if (nxt) load(kk + 1);
      compute(buf);
      if (nxt) {
        transform();
        store(buf ^ 1);
      }
      __syncthreads();
    }
  }

  // ------------------------------------------------------------ epilogue
  const int K = d.K;
  if constexpr (!GNA) {
  if (d.splits > 1 && d.tickets) {
    // Split-K combined inside the launch (the protocol of csrc/conv_halo9.hip / conv_small.hip: MI355X_MICROARCH.md,
    // inter-workgroup visibility, a counter hand-off with a write-through payload).  Each part stores its
    // accumulators in their register layout (16-byte pieces [part][i][j][thread] of the tile's slab of d.ws, sc1),
    // drains, one lane takes the tile's ticket; the part drawing the last one resets it, sums the parts in part order
    // (its own from registers) and runs the unsplit epilogue below.  The launcher admits whole tiles only.
    constexpr int SLOT = TM * TN * 4;   // floats per thread and part
    const auto rs = __builtin_amdgcn_make_buffer_rsrc(d.ws + (size_t)b * d.splits * NT * SLOT, 0,
                                                      d.splits * NT * SLOT * 4, 0x00020000);
    auto piece = [&](int s, int i, int j) { return (((s * TM + i) * TN + j) * NT + tid) * 16; };
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i][j]), rs, piece(split, i, j), 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    int* const last = (int*)lds;   // the staging buffers are dead after the main loop; the epilogue does not use them
    if (tid == 0) {
      auto* tk = (__attribute__((address_space(1))) unsigned*)(d.tickets + b);
      const unsigned t = __hip_atomic_fetch_add(tk, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      const int is_last = t == (unsigned)(d.splits - 1);
      if (is_last) __hip_atomic_store(tk, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      *last = is_last;
    }
    __syncthreads();
    if (!*last) return;
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    f32x4 tot[TM][TN];
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) tot[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll 1
    for (int s = 0; s < d.splits; ++s) {
      if (s == split) {
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) tot[i][j] += acc[i][j];
      } else {
        u32x4 v[TM][TN];
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) v[i][j] = __builtin_amdgcn_raw_buffer_load_b128(rs, piece(s, i, j), 0, 16);
#pragma unroll
        for (int i = 0; i < TM; ++i)
#pragma unroll
          for (int j = 0; j < TN; ++j) tot[i][j] += __builtin_bit_cast(f32x4, v[i][j]);
      }
    }
#pragma unroll
    for (int i = 0; i < TM; ++i)
#pragma unroll
      for (int j = 0; j < TN; ++j) acc[i][j] = tot[i][j];
  }
  }
  if (d.splits > 1 && !(!GNA && d.tickets)) {
    float* ws = d.ws + (size_t)split * A.Mfull * K;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int co = co0 + wm * (BCO / WM) + 16 * i + 4 * lq;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int pt = px0 + wn * (BPX / WN) + 16 * j + l16;
        if (pt >= A.M) continue;
        const int p = pmap(pt);
        float* dst = ws + (size_t)p * K + co;
        if (co + 3 < K) {
          *(f32x4*)dst = acc[i][j];
        } else {
          for (int r = 0; r < 4; ++r)
            if (co + r < K) dst[r] = acc[i][j][r];
        }
      }
    }
    return;
  }

  if (GNA) {
    // dx = acc + P*dz + Q*x + R (+ dx): the 1x1 skip-conv data gradient fused into the GroupNorm
    // backward of the same ResBlock input (gn_bwd_apply with extra = this conv's output, which is
    // rounded to bf16 exactly as that path stored it).  The tile goes through LDS so every global
    // access below is a coalesced 16-byte one (16 threads = one pixel's 128 channels).
    static_assert(BPX * BCO * 2 <= 2 * (BCO + BPX) * BK * 2, "GNA tile fits the staging LDS");
    const fmd_gn_apply_desc& g = A.g;
    const int C = K, C0 = g.C0, C1 = K - g.C0;
    bf16r* tile = lds;   // [BPX][BCO] bf16, 16-byte chunk index ^ (pixel & 15)
    constexpr int CHT = BCO / 8;
#pragma unroll
    for (int i = 0; i < TM; ++i) {
      const int cl = wm * (BCO / WM) + 16 * i + 4 * lq;
#pragma unroll
      for (int j = 0; j < TN; ++j) {
        const int pi = wn * (BPX / WN) + 16 * j + l16;
        u32x2 o;
        o[0] = pack2(acc[i][j][0], acc[i][j][1]);
        o[1] = pack2(acc[i][j][2], acc[i][j][3]);
        *(u32x2*)(tile + pi * BCO + (((cl >> 3) ^ (pi & (CHT - 1))) * 8) + (cl & 7)) = o;
      }
    }
    __syncthreads();
    const int c16 = tid % CHT;
    const int co = co0 + c16 * 8;
    if (co < K) {
      const bool first = co < C0;   // C0 % 8 == 0: the 8 channels are in one source
      const int accf = first ? g.acc0 : g.acc1;
      // HBM-bound: all of a thread's 16-byte reads (dz, x, old dx) are issued before any store, so each
      // thread keeps 16-24 reads in flight instead of the 2-deep unroll it had (measured 3.7 TB/s)
      constexpr int NQ = BPX * CHT / 256;
      constexpr int NB = NQ < 2 ? NQ : 2;   // pieces per batch: 6 reads in flight within the main loop's VGPRs
      static_assert(NQ * 256 == BPX * CHT && NQ % NB == 0, "GNA epilogue pieces per thread");
#pragma unroll 1
      for (int k0 = 0; k0 < NQ; k0 += NB) {
      u32x4 vz[NB], vx[NB], old[NB];
#pragma unroll
      for (int kk = 0; kk < NB; ++kk) {
        const int k = kk;
        const int pi = (tid + 256 * (k0 + kk)) / CHT;
        const int p = min(px0 + pi, A.M - 1);   // rows past M: clamped reads, no store
        vz[k] = *(const u32x4*)((const bf16r*)g.dz + (size_t)p * C + co);
        vx[k] = first ? *(const u32x4*)((const bf16r*)g.x0 + (size_t)p * C0 + co)
                      : *(const u32x4*)((const bf16r*)g.x1 + (size_t)p * C1 + (co - C0));
        old[k] = u32x4{0u, 0u, 0u, 0u};
        if (accf)
          old[k] = first ? *(const u32x4*)((const bf16r*)g.dx0 + (size_t)p * C0 + co)
                         : *(const u32x4*)((const bf16r*)g.dx1 + (size_t)p * C1 + (co - C0));
      }
#pragma unroll
      for (int k = 0; k < NB; ++k) {
        const int pi = (tid + 256 * (k0 + k)) / CHT;
        const int p = px0 + pi;
        if (p >= A.M) continue;
        const int n = p / HWo;
        const u32x4 ve = *(const u32x4*)(tile + pi * BCO + ((c16 ^ (pi & (CHT - 1))) * 8));
        bf16r* dst = first ? (bf16r*)g.dx0 + (size_t)p * C0 + co : (bf16r*)g.dx1 + (size_t)p * C1 + (co - C0);
        const float* pp = g.P + (size_t)n * C + co;
        const float* qq = g.Q + (size_t)n * C + co;
        const float* rr = g.R + (size_t)n * C + co;
        const f32x4 P0 = *(const f32x4*)pp, P1 = *(const f32x4*)(pp + 4);
        const f32x4 Q0 = *(const f32x4*)qq, Q1 = *(const f32x4*)(qq + 4);
        const f32x4 R0 = *(const f32x4*)rr, R1 = *(const f32x4*)(rr + 4);
        const float Pv[8] = {P0[0], P0[1], P0[2], P0[3], P1[0], P1[1], P1[2], P1[3]};
        const float Qv[8] = {Q0[0], Q0[1], Q0[2], Q0[3], Q1[0], Q1[1], Q1[2], Q1[3]};
        const float Rv[8] = {R0[0], R0[1], R0[2], R0[3], R1[0], R1[1], R1[2], R1[3]};
        u32x4 o;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          float lo = Pv[2 * e] * bf_lo(vz[k][e]) + Qv[2 * e] * bf_lo(vx[k][e]) + Rv[2 * e] + bf_lo(ve[e]);
          float hi = Pv[2 * e + 1] * bf_hi(vz[k][e]) + Qv[2 * e + 1] * bf_hi(vx[k][e]) + Rv[2 * e + 1] +
                     bf_hi(ve[e]);
          if (accf) { lo += bf_lo(old[k][e]); hi += bf_hi(old[k][e]); }
          o[e] = pack2(lo, hi);
        }
        *(u32x4*)dst = o;
      }
      }
    }
    return;
  }

  const bool stats = d.stats != nullptr;
  const bool dep = d.ep_a != nullptr;
  const bool hasx = d.ep_x0 != nullptr;
  float st1[TM][4], st2[TM][4];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int r = 0; r < 4; ++r) { st1[i][r] = 0.f; st2[i][r] = 0.f; }

#pragma unroll
  for (int i = 0; i < TM; ++i) {
    const int co = co0 + wm * (BCO / WM) + 16 * i + 4 * lq;
    if (co >= K) continue;
    const bool full = co + 3 < K;
    float bias[4] = {0.f, 0.f, 0.f, 0.f};
    if (d.bias) {
      for (int r = 0; r < 4; ++r) bias[r] = (co + r < K) ? d.bias[co + r] : 0.f;
    }
    if (d.bias2) {
      for (int r = 0; r < 4; ++r) bias[r] += (co + r < K) ? d.bias2[co + r] : 0.f;
    }
#pragma unroll
    for (int j = 0; j < TN; ++j) {
      const int pt = px0 + wn * (BPX / WN) + 16 * j + l16;
      if (pt >= A.M) continue;
      const int p = pmap(pt);
      const int n = p / HWo;
      float v[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) v[r] = acc[i][j][r] + bias[r];
      if (d.bias_nc) {
        for (int r = 0; r < 4; ++r)
          if (co + r < K) v[r] += d.bias_nc[(size_t)n * K + co + r];
      }
      if (d.resid) {
        const bf16r* rp = (const bf16r*)d.resid + (size_t)p * K + co;
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
        // data-gradient epilogue: dz = d(act) * silu'(a*x + b), x = forward GN input
        const int C0e = d.ep_C0;
        for (int r = 0; r < 4; ++r) {
          const int c = co + r;
          if (c >= K) continue;
          const bf16r* xp = (c < C0e) ? (const bf16r*)d.ep_x0 + (size_t)p * C0e + c
                                      : (const bf16r*)d.ep_x1 + (size_t)p * (K - C0e) + (c - C0e);
          const float x = bf2f(*xp);
          xv[r] = x;
          if (dep) {
            const float z = d.ep_a[(size_t)n * K + c] * x + d.ep_b[(size_t)n * K + c];
            v[r] *= silu_grad(z);
          }
        }
      }
      if (d.out_f32) {
        float* op = (float*)d.out + (size_t)p * K + co;
        for (int r = 0; r < 4; ++r)
          if (co + r < K) op[r] = d.accumulate ? op[r] + v[r] : v[r];
      } else {
        bf16r* op = (bf16r*)d.out + (size_t)p * K + co;
        if (full) {
          if (d.accumulate) {
            const u32x2 o = *(const u32x2*)op;
            v[0] += bf_lo(o[0]); v[1] += bf_hi(o[0]); v[2] += bf_lo(o[1]); v[3] += bf_hi(o[1]);
          }
          u32x2 o;
          o[0] = pack2(v[0], v[1]);
          o[1] = pack2(v[2], v[3]);
          *(u32x2*)op = o;
          // statistics are taken on the rounded values the consumer will read
          v[0] = bf_lo(o[0]); v[1] = bf_hi(o[0]); v[2] = bf_lo(o[1]); v[3] = bf_hi(o[1]);
        } else {
          for (int r = 0; r < 4; ++r)
            if (co + r < K) {
              float w = d.accumulate ? bf2f(op[r]) + v[r] : v[r];
              op[r] = (bf16r)f2bf(w);
              v[r] = bf2f(op[r]);
            }
        }
      }
      if (stats) {
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          st1[i][r] += v[r];
          st2[i][r] += hasx ? v[r] * xv[r] : v[r] * v[r];
        }
      }
    }
  }
  if (stats) {
    // reduce over the 16 pixel lanes of each quad-row; the wave's pixels are one image.  Parity classes:
    // rows stay image-major (image n owns rows [n HW/64, (n+1) HW/64)), class c the c-th HWq/64 of them --
    // a class row holds strided pixels, which GroupNorm's per-(image, channel) sums do not mind
    const int pw = px0 + wn * (BPX / WN);
    int srow = pw / A.stats_rows;
    if (A.par) {
      const int ncls = d3 ? 8 : 4, cls = (int)blockIdx.z, rpi = HWq / A.stats_rows;
      const int n = pw / HWq;
      srow = (n * ncls + cls) * rpi + (pw - n * HWq) / A.stats_rows;
    }
#pragma unroll
    for (int i = 0; i < TM; ++i) {
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        float a = st1[i][r], q = st2[i][r];
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
          a += __shfl_xor(a, o, 64);
          q += __shfl_xor(q, o, 64);
        }
        const int co = co0 + wm * (BCO / WM) + 16 * i + 4 * lq + r;
        if (l16 == 0 && co < K) {
          float* sp = d.stats + ((size_t)srow * K + co) * 2;
          sp[0] = a;
          sp[1] = q;
        }
      }
    }
  }
}

__global__ void splitk_reduce(const fmd_conv_desc d, int M) {
  const int K = d.K;
  const int HWo = (d.Do > 0 ? d.Do : 1) * d.Ho * d.Wo;
  const size_t total = (size_t)M * K;
  for (size_t idx = (size_t)blockIdx.x * blockDim.x + threadIdx.x; idx < total; idx += (size_t)gridDim.x * blockDim.x) {
    const int p = (int)(idx / K);
    const int c = (int)(idx - (size_t)p * K);
    const int n = p / HWo;
    // the tiny levels split K 16-72 ways: 8 independent loads in flight per thread, not one chain
    float a8[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    int s = 0;
    for (; s + 8 <= d.splits; s += 8) {
#pragma unroll
      for (int u = 0; u < 8; ++u) a8[u] += d.ws[(size_t)(s + u) * total + idx];
    }
    for (; s < d.splits; ++s) a8[0] += d.ws[(size_t)s * total + idx];
    float v = ((a8[0] + a8[1]) + (a8[2] + a8[3])) + ((a8[4] + a8[5]) + (a8[6] + a8[7]));
    if (d.bias) v += d.bias[c];
    if (d.bias2) v += d.bias2[c];
    if (d.bias_nc) v += d.bias_nc[(size_t)n * K + c];
    if (d.resid) v += bf2f(((const bf16r*)d.resid)[idx]);
    if (d.ep_a) {
      const int C0e = d.ep_C0;
      const float x = (c < C0e) ? bf2f(((const bf16r*)d.ep_x0)[(size_t)p * C0e + c])
                                : bf2f(((const bf16r*)d.ep_x1)[(size_t)p * (K - C0e) + (c - C0e)]);
      v *= silu_grad(d.ep_a[(size_t)n * K + c] * x + d.ep_b[(size_t)n * K + c]);
    }
    if (d.out_f32) {
      float* o = (float*)d.out + idx;
      *o = d.accumulate ? *o + v : v;
    } else {
      bf16r* o = (bf16r*)d.out + idx;
      *o = (bf16r)f2bf(d.accumulate ? bf2f(*o) + v : v);
    }
  }
}

// Split-K combine over 16-pixel rows x 64-channel blocks, one pixel x 4 channels per lane (16-byte slab
// loads), with the same epilogue as splitk_reduce and, when d.stats is set, the channel statistics of the
// rounded output (sum v, sum v^2 -- or sum v*x with the data-gradient epilogue) written as slab row p/16
// (FMD_SPLIT_STATS_ROWS), so no separate statistics pass is needed.  Split-K only runs on the small
// levels: 16-pixel rows give enough blocks there.  Needs K % 4 == 0 and M % 16 == 0.
__global__ __launch_bounds__(256) void splitk_reduce_rows(const fmd_conv_desc d, int M) {
  const int K = d.K;
  const int HWo = (d.Do > 0 ? d.Do : 1) * d.Ho * d.Wo;
  const size_t total = (size_t)M * K;
  constexpr int RP = FMD_SPLIT_STATS_ROWS;
  const int row = blockIdx.x;
  const int tq = threadIdx.x & 15, pl = threadIdx.x >> 4;
  static_assert(RP == 16, "one pixel per 16-lane group");
  const int c = blockIdx.y * 64 + tq * 4;
  const bool cok = c < K;
  const bool hasx = d.ep_x0 != nullptr;
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  if (cok) {
    {
      const int p = row * RP + pl;
      const int n = p / HWo;
      const size_t idx = (size_t)p * K + c;
      // four independent chains over the splits (loads of four slabs in flight), fixed summation order
      f32x4 v = *(const f32x4*)(d.ws + idx), v1 = {0.f, 0.f, 0.f, 0.f}, v2 = v1, v3 = v1;
      int s = 1;
      for (; s + 4 <= d.splits; s += 4) {
        v += *(const f32x4*)(d.ws + (size_t)s * total + idx);
        v1 += *(const f32x4*)(d.ws + (size_t)(s + 1) * total + idx);
        v2 += *(const f32x4*)(d.ws + (size_t)(s + 2) * total + idx);
        v3 += *(const f32x4*)(d.ws + (size_t)(s + 3) * total + idx);
      }
      for (; s < d.splits; ++s) v += *(const f32x4*)(d.ws + (size_t)s * total + idx);
      v = (v + v1) + (v2 + v3);
      if (d.bias) v += *(const f32x4*)(d.bias + c);
      if (d.bias2) v += *(const f32x4*)(d.bias2 + c);
      if (d.bias_nc) {   // may be a row view of a wider table: no 16-byte alignment assumed
        const float* bn = d.bias_nc + (size_t)n * K + c;
        v += f32x4{bn[0], bn[1], bn[2], bn[3]};
      }
      if (d.resid) {
        const u32x2 r = *(const u32x2*)((const bf16r*)d.resid + idx);
        v[0] += bf_lo(r[0]); v[1] += bf_hi(r[0]); v[2] += bf_lo(r[1]); v[3] += bf_hi(r[1]);
      }
      float xv[4] = {0.f, 0.f, 0.f, 0.f};
      if (hasx) {
        const int C0e = d.ep_C0;
        const u32x2 r = c < C0e ? *(const u32x2*)((const bf16r*)d.ep_x0 + (size_t)p * C0e + c)
                                : *(const u32x2*)((const bf16r*)d.ep_x1 + (size_t)p * (K - C0e) + (c - C0e));
        xv[0] = bf_lo(r[0]); xv[1] = bf_hi(r[0]); xv[2] = bf_lo(r[1]); xv[3] = bf_hi(r[1]);
        if (d.ep_a) {
          const f32x4 ea = *(const f32x4*)(d.ep_a + (size_t)n * K + c), eb = *(const f32x4*)(d.ep_b + (size_t)n * K + c);
#pragma unroll
          for (int r2 = 0; r2 < 4; ++r2) v[r2] *= silu_grad(ea[r2] * xv[r2] + eb[r2]);
        }
      }
      if (d.out_f32) {
        f32x4* o = (f32x4*)((float*)d.out + idx);
        *o = d.accumulate ? *o + v : v;
      } else {
        u32x2* o = (u32x2*)((bf16r*)d.out + idx);
        if (d.accumulate) {
          const u32x2 old = *o;
          v[0] += bf_lo(old[0]); v[1] += bf_hi(old[0]); v[2] += bf_lo(old[1]); v[3] += bf_hi(old[1]);
        }
        u32x2 w;
        w[0] = pack2(v[0], v[1]);
        w[1] = pack2(v[2], v[3]);
        *o = w;
        const float wr[4] = {bf_lo(w[0]), bf_hi(w[0]), bf_lo(w[1]), bf_hi(w[1])};
#pragma unroll
        for (int r2 = 0; r2 < 4; ++r2) {
          s1[r2] += wr[r2];
          s2[r2] += hasx ? wr[r2] * xv[r2] : wr[r2] * wr[r2];
        }
      }
    }
  }
  if (!d.stats) return;
  // lanes tq, tq+16, tq+32, tq+48 of a wave hold the same channels (4 pixels); then the 4 waves via LDS
  __shared__ float red[4][64][2];
#pragma unroll
  for (int r2 = 0; r2 < 4; ++r2) {
    s1[r2] += __shfl_xor(s1[r2], 16, 64);
    s1[r2] += __shfl_xor(s1[r2], 32, 64);
    s2[r2] += __shfl_xor(s2[r2], 16, 64);
    s2[r2] += __shfl_xor(s2[r2], 32, 64);
  }
  const int wv = threadIdx.x >> 6;
  if ((threadIdx.x & 63) < 16) {
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) { red[wv][tq * 4 + r2][0] = s1[r2]; red[wv][tq * 4 + r2][1] = s2[r2]; }
  }
  __syncthreads();
  if (threadIdx.x < 128) {
    const int cl = threadIdx.x >> 1, k = threadIdx.x & 1;
    const int cc = blockIdx.y * 64 + cl;
    if (cc < K)
      d.stats[((size_t)row * K + cc) * 2 + k] = (red[0][cl][k] + red[1][cl][k]) + (red[2][cl][k] + red[3][cl][k]);
  }
}

// Split-K combine + the GroupNorm forward of the result: a 1024-thread block owns (image n, CB channels) with
// CB = max(CONV_GN_CB (default 4; fmd_conv_gn_set_block_channels), Cg) -- whole groups, so the group statistics close inside it.  Pass 1: lanes = (4-channel quad,
// pixel lane) over the image's pixels (slab sums in four chains, fixed order), bias / per-sample bias / residual,
// bf16 out, and the channel sums of the rounded values; lanes (shuffles), waves (LDS) and the group's channels
// (fp64) in fixed order; pass 2 writes t = SiLU(a*out + b) from the lane's own output elements (the first pixel's
// kept in registers, later ones re-read).
constexpr int CGN_NT = 1024;
__global__ __launch_bounds__(CGN_NT) void combine_gn_kernel(const fmd_conv_desc d, const fmd_gn_out_desc g, int M,
                                                            int CB) {
  const int K = d.K;
  const int HW = (d.Do > 0 ? d.Do : 1) * d.Ho * d.Wo;
  const size_t total = (size_t)M * K;
  const int n = blockIdx.x, cb = blockIdx.y * CB;
  const int nq = CB / 4, PL = CGN_NT / nq;
  const int tq = threadIdx.x % nq, pl = threadIdx.x / nq;
  const int c = cb + tq * 4;
  f32x4 add = {0.f, 0.f, 0.f, 0.f};
  if (d.bias) add += *(const f32x4*)(d.bias + c);
  if (d.bias2) add += *(const f32x4*)(d.bias2 + c);
  if (d.bias_nc) {
    const float* bn = d.bias_nc + (size_t)n * K + c;
    add += f32x4{bn[0], bn[1], bn[2], bn[3]};
  }
  float s1[4] = {0.f, 0.f, 0.f, 0.f}, s2[4] = {0.f, 0.f, 0.f, 0.f};
  u32x2 wkeep = {0u, 0u};   // the lane's first pixel's output, kept for pass 2 (on the small levels its only one)
  for (int pp = pl; pp < HW; pp += PL) {
    const size_t idx = ((size_t)n * HW + pp) * K + c;
    f32x4 v = *(const f32x4*)(d.ws + idx), v1 = {0.f, 0.f, 0.f, 0.f}, v2 = v1, v3 = v1;
    int s = 1;
    for (; s + 4 <= d.splits; s += 4) {
      v += *(const f32x4*)(d.ws + (size_t)s * total + idx);
      v1 += *(const f32x4*)(d.ws + (size_t)(s + 1) * total + idx);
      v2 += *(const f32x4*)(d.ws + (size_t)(s + 2) * total + idx);
      v3 += *(const f32x4*)(d.ws + (size_t)(s + 3) * total + idx);
    }
    for (; s < d.splits; ++s) v += *(const f32x4*)(d.ws + (size_t)s * total + idx);
    v = ((v + v1) + (v2 + v3)) + add;
    if (d.resid) {
      const u32x2 r = *(const u32x2*)((const bf16r*)d.resid + idx);
      v[0] += bf_lo(r[0]); v[1] += bf_hi(r[0]); v[2] += bf_lo(r[1]); v[3] += bf_hi(r[1]);
    }
    u32x2 w;
    w[0] = pack2(v[0], v[1]);
    w[1] = pack2(v[2], v[3]);
    *(u32x2*)((bf16r*)d.out + idx) = w;
    if (pp == pl) wkeep = w;
    const float wr[4] = {bf_lo(w[0]), bf_hi(w[0]), bf_lo(w[1]), bf_hi(w[1])};
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) {
      s1[r2] += wr[r2];
      s2[r2] += wr[r2] * wr[r2];
    }
  }
  // lanes of one wave holding the same quad sit nq apart: butterfly over those, then the 16 waves via LDS
  for (int o = nq; o < 64; o <<= 1) {
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) {
      s1[r2] += __shfl_xor(s1[r2], o, 64);
      s2[r2] += __shfl_xor(s2[r2], o, 64);
    }
  }
  __shared__ float red[CGN_NT / 64][64][2];
  __shared__ float chs[64][2];
  __shared__ double gst[64][2];   // ng = CB / Cg groups per block: up to 64 (CB <= 64, Cg >= 1)
  __shared__ float ab[64][2];
  const int wv = threadIdx.x >> 6, ln = threadIdx.x & 63;
  if (ln < nq) {
#pragma unroll
    for (int r2 = 0; r2 < 4; ++r2) { red[wv][ln * 4 + r2][0] = s1[r2]; red[wv][ln * 4 + r2][1] = s2[r2]; }
  }
  __syncthreads();
  if (threadIdx.x < 2 * CB) {   // per channel over the 16 waves
    const int cl = threadIdx.x >> 1, k = threadIdx.x & 1;
    float a0 = 0.f, a1 = 0.f;
#pragma unroll
    for (int w2 = 0; w2 < CGN_NT / 64; w2 += 2) { a0 += red[w2][cl][k]; a1 += red[w2 + 1][cl][k]; }
    chs[cl][k] = a0 + a1;
  }
  __syncthreads();
  const int Cg = K / g.G, ng = CB / Cg;
  if (threadIdx.x < ng) {   // group sums in fp64 over its Cg channels, E[x^2] - mean^2 (as gn_fused_apply)
    double t1 = 0.0, t2 = 0.0;
    for (int cl = threadIdx.x * Cg; cl < (threadIdx.x + 1) * Cg; ++cl) {
      t1 += (double)chs[cl][0];
      t2 += (double)chs[cl][1];
    }
    const double cnt = (double)Cg * HW;
    const double mean = t1 / cnt;
    double var = t2 / cnt - mean * mean;
    if (var < 0) var = 0;
    const double rstd = 1.0 / sqrt(var + (double)g.eps);
    gst[threadIdx.x][0] = mean;
    gst[threadIdx.x][1] = rstd;
    const int gi = cb / Cg + threadIdx.x;
    g.mean_rstd[((size_t)n * g.G + gi) * 2] = (float)mean;
    g.mean_rstd[((size_t)n * g.G + gi) * 2 + 1] = (float)rstd;
  }
  __syncthreads();
  if (threadIdx.x < CB) {
    const int cc = cb + threadIdx.x, gl = threadIdx.x / Cg;
    const float meanf = (float)gst[gl][0], rstd = (float)gst[gl][1];
    const float gm = g.gamma ? g.gamma[cc] : 1.f, bt = g.beta ? g.beta[cc] : 0.f;
    float av = rstd * gm;
    float bv = bt - meanf * av;
    if (g.emb_mode == 1) {
      const float sc = 1.f + g.emb[(size_t)n * g.emb_stride + cc];
      const float sh = g.emb[(size_t)n * g.emb_stride + K + cc];
      av *= sc;
      bv = bv * sc + sh;
    }
    ab[threadIdx.x][0] = av;
    ab[threadIdx.x][1] = bv;
    g.a[(size_t)n * K + cc] = av;
    g.b[(size_t)n * K + cc] = bv;
  }
  __syncthreads();
  float av[4], bv[4];
#pragma unroll
  for (int r2 = 0; r2 < 4; ++r2) { av[r2] = ab[tq * 4 + r2][0]; bv[r2] = ab[tq * 4 + r2][1]; }
  for (int pp = pl; pp < HW; pp += PL) {   // the lane's own pass-1 stores: program order makes them visible
    const size_t idx = ((size_t)n * HW + pp) * K + c;
    const u32x2 w = pp == pl ? wkeep : *(const u32x2*)((const bf16r*)d.out + idx);
    float y[4] = {bf_lo(w[0]) * av[0] + bv[0], bf_hi(w[0]) * av[1] + bv[1], bf_lo(w[1]) * av[2] + bv[2],
                  bf_hi(w[1]) * av[3] + bv[3]};
    if (g.silu) {
#pragma unroll
      for (int r2 = 0; r2 < 4; ++r2) y[r2] = siluf_(y[r2]);
    }
    u32x2 o;
    o[0] = pack2(y[0], y[1]);
    o[1] = pack2(y[2], y[3]);
    *(u32x2*)((bf16r*)g.t + idx) = o;
  }
}

template <int BCO, int BPX, int WM, int WN, int BK, bool GNA = false>
int launch(const fmd_conv_desc* d, hipStream_t s, const fmd_gn_apply_desc* g = nullptr) {
  KArgs A;
  A.d = *d;
  if (g) A.g = *g;
  const int Dz = d->Do > 0 ? d->Do : 1;
  A.M = d->N * Dz * d->Ho * d->Wo;
  A.T = d->ks * d->ks * (d->Do > 0 ? d->ks : 1);
  A.C = d->C0 + d->C1;
  A.pack = A.C == 8 && BK >= 16 && !GNA;
  A.nk1 = A.pack ? (A.T + BK / 8 - 1) / (BK / 8) : ((A.C + BK - 1) / BK) * A.T;
  A.nk = A.nk1 + (d->src2 ? (d->C2 + d->C3 + BK - 1) / BK : 0);
  const int splits = d->splits > 1 ? d->splits : 1;
  A.per_split = (A.nk + splits - 1) / splits;
  A.Mfull = A.M;
  // parity classes; with fused statistics every class must tile its images by whole 64-pixel rows
  const int HWq = (d->Do > 0 ? d->Do / 2 : 1) * (d->Ho / 2) * (d->Wo / 2);
  A.par = d->transposed && d->stride == 2 && d->ks == 3 && d->pad == 1 && !(d->Ho & 1) && !(d->Wo & 1) &&
          !(d->Do & 1) && (!d->stats || (HWq % 64 == 0 && (d->N * HWq) % BPX == 0)) && !d->src2 && !GNA && !A.pack;
  if (A.par) A.M = d->N * (d->Do > 0 ? d->Do / 2 : 1) * (d->Ho / 2) * (d->Wo / 2);   // pixels per parity class
  A.ntp = (A.M + BPX - 1) / BPX;
  A.ntc = (d->K + BCO - 1) / BCO;
  A.stats_rows = 64;
  // split-K combined inside the launch (d->tickets): whole tiles, no parity classes; the statistics then come from the
  // unsplit epilogue with one row per wave's pixel range (BPX / WN pixels)
  const bool tk = splits > 1 && d->tickets;
  if (tk && (GNA || A.par || A.M % BPX || d->K % BCO || d->out_f32 || d->accumulate ||
             d->n_tickets < A.ntp * A.ntc))
    return -14;
  if (d->stats) {
    // every wave's pixel range must be one image and full
    const int wrows = BPX / WN;
    if (tk) {
      if ((Dz * d->Ho * d->Wo) % wrows != 0 || d->tickets_rows != wrows) return -14;
      A.stats_rows = wrows;
    } else if (wrows != 64 || (Dz * d->Ho * d->Wo) % 64 != 0 || A.M % BPX != 0 || splits > 1 || (A.par && HWq % 64)) {
      return -11;
    }
  }
  dim3 grid(A.ntp * A.ntc, splits, A.par ? (d->Do > 0 ? 8 : 4) : 1);
  hipLaunchKernelGGL((conv_igemm<BCO, BPX, WM, WN, BK, GNA>), grid, dim3(256), 0, s, A);
  return (int)hipGetLastError();
}

}  // namespace

// combine = false: the split-K partial slabs only (fmd_conv_gn runs its own combine)
static int conv_run(const fmd_conv_desc* d, fmd_stream_t stream, bool combine) {
  hipStream_t s = (hipStream_t)stream;
  // largest output (pixels) run on 64- / 32-pixel tiles when split-K (mirrored by ops.BPX64_M / BPX32_M)
  constexpr int small_m = 2048, tiny_m = 128;
  const int C = d->C0 + d->C1;
  if ((d->C0 % 8) || (d->C1 % 8) || (d->C2 % 8) || (d->C3 % 8) || d->ks < 1 || d->N < 1) return -1;
  if (d->C3 && !d->src3) return -6;
  if (d->C1 && !d->src1) return -2;
  if (d->src2 && !d->wgt2 && !d->wgt2_tiled) return -3;
  if (d->pro_a && !d->pro_b) return -4;
  if (d->gout && !d->pro_a) return -9;
  const int M = d->N * (d->Do > 0 ? d->Do : 1) * d->Ho * d->Wo;
  const int HWo = (d->Do > 0 ? d->Do : 1) * d->Ho * d->Wo;
  // split-K: the combine kernel produces the channel statistics (16-pixel rows) instead of the main kernel
  const bool rows_ok = d->K % 4 == 0 && M % FMD_SPLIT_STATS_ROWS == 0 && HWo % FMD_SPLIT_STATS_ROWS == 0;
  if (d->splits > 1 && (!d->ws || (d->stats && (!rows_ok || d->out_f32 || d->accumulate)))) return -5;
  (void)C;
  fmd_conv_desc dm = *d;
  const bool tk = d->splits > 1 && d->tickets && combine;   // split-K combined inside the launch
  if (!tk) dm.tickets = nullptr;
  if (d->splits > 1 && !tk) dm.stats = nullptr;
  int rc = 1;
  if (d->K > 16 && !d->force_generic)
    rc = fmd_conv_halo(&dm, stream);   // 3x3 stride-1 problems with >= HALO_MIN_WG (32) workgroups of 16x16 tiles (x splits)
  if (rc == 1 && d->fold_st0) return -13;   // the in-kernel GroupNorm fold runs only on the halo kernel
  // a ticketed problem the halo kernel declined runs ticketed on the implicit GEMM, or not at all (-14: the caller
  // splits the two-launch way; the statistics' row size differs)
  if (rc == 1 && tk && (!d->wgt || (d->src2 && !d->wgt2) || d->gout)) return -14;
  if (rc == 1) {
    if (!d->wgt || (d->src2 && !d->wgt2)) return -8;   // only halo tiles were supplied, but the halo path declined
    if (d->gout) return -9;                            // the prologue side output exists only on the halo path
    if (d->K <= 16)
      rc = launch<16, 256, 1, 4, 64>(&dm, s);
    else if (d->K <= 64)
      rc = launch<64, 128, 2, 2, 64>(&dm, s);
    else if (M <= tiny_m && d->splits > 1)    // tinier: 32-pixel tiles
      rc = launch<128, 32, 2, 2, 64>(&dm, s);
    else if (M <= small_m && d->splits > 1)   // tiny levels: 64-pixel tiles, half the split-K slabs
      rc = launch<128, 64, 2, 2, 64>(&dm, s);
    else
      rc = launch<128, 128, 2, 2, 64>(&dm, s);
  }
  if (rc) return rc;
  if (d->splits > 1 && combine && !tk) {
    if (rows_ok) {
      hipLaunchKernelGGL(splitk_reduce_rows, dim3(M / FMD_SPLIT_STATS_ROWS, (d->K + 63) / 64), dim3(256), 0, s, *d, M);
    } else {
      const size_t total = (size_t)M * d->K;
      int blocks = (int)((total + 255) / 256);
      if (blocks > 8192) blocks = 8192;
      hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, s, *d, M);
    }
    rc = (int)hipGetLastError();
  }
  return rc;
}

extern "C" int fmd_conv(const fmd_conv_desc* d, fmd_stream_t stream) { return conv_run(d, stream, true); }

static int g_conv_gn_cb = 4;   // fmd_conv_gn_set_block_channels (runtime/tuning.py CONV_GN_CB)
static int conv_gn_cb() { return g_conv_gn_cb; }

extern "C" int fmd_conv_gn_set_block_channels(int32_t cb) {
  if (cb != 4 && cb != 8 && cb != 16 && cb != 32 && cb != 64) return -1;
  g_conv_gn_cb = cb;
  return 0;
}

extern "C" int fmd_conv_gn(const fmd_conv_desc* d, const fmd_gn_out_desc* g, fmd_stream_t stream) {
  if (!g || !g->a || !g->b || !g->mean_rstd || !g->t || g->G < 1 || d->K % g->G) return -12;
  const int Cg = d->K / g->G;
  if (d->splits < 2 || d->K % 64 || 64 % Cg || d->stats || d->out_f32 || d->accumulate || d->ep_x0 || d->ep_a)
    return -12;
  // channels per block: whole groups, at least CONV_GN_CB (default 4: one quad x 1024 pixel lanes when a group
  // is 4 channels -- more blocks on the 128-channel levels; latent sampler 82.3 / 82.6 (16) -> 81.8 / 82.0 (8)
  // -> 81.3 / 81.5 ms (4), interleaved A/B)
  const int cb_min = conv_gn_cb();
  const int CB = Cg > cb_min ? Cg : cb_min;
  if (g->emb_mode == 1 && !g->emb) return -12;
  if (!d->ws || d->N < 1) return -12;
  int rc = conv_run(d, stream, false);
  if (rc) return rc;
  const int M = d->N * (d->Do > 0 ? d->Do : 1) * d->Ho * d->Wo;
  hipLaunchKernelGGL(combine_gn_kernel, dim3(d->N, d->K / CB), dim3(CGN_NT), 0, (hipStream_t)stream, *d, *g, M, CB);
  return (int)hipGetLastError();
}

// The split-K combine alone: out = sum of d->splits fp32 slabs in d->ws ([splits][M][K]) + the conv
// epilogue (bias, bias2, per-sample bias, residual, data-gradient SiLU' / GN-backward sums, statistics).
// Used by convolutions assembled from several partial launches (3-D convs as three depth-tap planes).
extern "C" int fmd_conv_combine(const fmd_conv_desc* d, fmd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if (!d->ws || d->splits < 1 || d->N < 1 || d->K < 1 || !d->out) return -1;
  const int M = d->N * (d->Do > 0 ? d->Do : 1) * d->Ho * d->Wo;
  const int HWo = (d->Do > 0 ? d->Do : 1) * d->Ho * d->Wo;
  const bool rows_ok = d->K % 4 == 0 && M % FMD_SPLIT_STATS_ROWS == 0 && HWo % FMD_SPLIT_STATS_ROWS == 0;
  if (d->stats && (!rows_ok || d->out_f32 || d->accumulate)) return -5;
  if (rows_ok) {
    hipLaunchKernelGGL(splitk_reduce_rows, dim3(M / FMD_SPLIT_STATS_ROWS, (d->K + 63) / 64), dim3(256), 0, s, *d, M);
  } else {
    const size_t total = (size_t)M * d->K;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(splitk_reduce, dim3(blocks), dim3(256), 0, s, *d, M);
  }
  return (int)hipGetLastError();
}

// 1x1 (or any generic-path) conv whose epilogue is the GroupNorm-backward apply of fmd_gn_bwd_apply:
// dx = conv(...) + P*dz + Q*x + R (+ dx), split over the concat sources at g->C0.  d: no split-K, no
// stats/bias/residual/out (the result only exists as dx).
extern "C" int fmd_conv_gn_apply(const fmd_conv_desc* d, const fmd_gn_apply_desc* g, fmd_stream_t stream) {
  hipStream_t s = (hipStream_t)stream;
  if ((d->C0 % 8) || (d->C1 % 8) || (d->C2 % 8) || (d->C3 % 8) || d->ks < 1 || d->N < 1) return -1;
  if (d->splits > 1 || d->stats || d->bias || d->bias2 || d->bias_nc || d->resid || d->ep_x0 || d->src2) return -5;
  if (!g || !g->dz || !g->x0 || !g->P || !g->Q || !g->R || !g->dx0 || (g->C0 % 8)) return -7;
  if (g->C0 < d->K && (!g->x1 || !g->dx1)) return -7;
  // BK = 32: a 32 KiB LDS footprint keeps 4-5 of these memory-bound workgroups per CU in flight
  if (d->K <= 64) return launch<64, 128, 2, 2, 32, true>(d, s, g);
  return launch<128, 128, 2, 2, 32, true>(d, s, g);
}
