// Softmax attention on MFMA (gfx950 v_mfma_f32_32x32x16_bf16): QK^T and PV (and the backward's dP, dS
// products) as matrix-core tiles with an fp32 online softmax -- the UNet / VAE self-attention blocks
// (SpatialSelfAttention's raw head split, DiffusersAttentionND's view/transpose split) and the
// cross-attention blocks (SpatialCrossAttention, DiffusersAttentionND with a context), replacing
// F.scaled_dot_product_attention (src/nn/blocks/attention.py:42-44, 115, 185, 269).
//
// Layout.  The head split of the reference (raw reshape or view/transpose, self or cross) is undone by
// fmd_attn_pack into canonical bf16 [B*heads][rows][DHP] planes (head dim zero-padded to DHP = 16, 32 or 64),
// so the MFMA kernels read 16-byte fragments; fmd_attn_unpack writes canonical results back through the
// same index map.
//
// Orientation.  The forward computes S^T = K Q^T (keys on the MFMA rows, queries on its columns = lanes):
// the softmax statistics of a query are then one lane's registers plus its partner half-wave, the
// rescale by exp(m_old - m_new) is a per-lane scalar, and P^T feeds the next product O^T += V^T P^T
// straight from the accumulator registers (registers 8s..8s+7 are k-step s, rows in the order
// 16s + 8(j>>2) + 4h + (j&3)); V^T fragments come from the [key][d] LDS block with ds_read_b64_tr_b16.
// Backward: dQ^T = K^T dS^T per query block (keys streamed), dV^T = dO^T P and dK^T = Q^T dS per key
// block (queries streamed), P recomputed from the saved log-sum-exp (flash-style, no T x T buffer).
#include "common.h"
#include "../../include/fmdiff.h"

namespace {

typedef __attribute__((ext_vector_type(16))) float f32x16;

FMD_DEV f32x16 mfma32(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

constexpr float LOG2E = 1.4426950408889634f;
constexpr float LN2 = 0.6931471805599453f;

// reference head split (same map as csrc/attention.hip AGeo): element (which, h, r, d) of one batch's buffer
struct Geo {
  int Tq, Tk, heads, dh, inner, raw, cross;
  FMD_HD int parts(int which) const { return which == 3 ? 1 : (cross ? (which ? 2 : 1) : 3); }
  FMD_HD int slot(int which) const { return which == 3 ? 0 : (cross && which ? which - 1 : which); }
  FMD_HD int rows(int which) const { return (which == 1 || which == 2) ? Tk : Tq; }
  FMD_DEV unsigned off(int which, int h, int r, int d) const {
    const unsigned P = parts(which), T = rows(which);
    if (raw) {
      const unsigned f = ((unsigned)h * T + r) * P * dh + slot(which) * dh + d;
      const unsigned c = f / T;
      return (f - c * T) * P * inner + c;
    }
    return (unsigned)r * P * inner + slot(which) * inner + h * dh + d;
  }
  FMD_HD size_t stride(int which) const { return (size_t)rows(which) * parts(which) * inner; }
};

// canonical plane of (which in {0 q, 1 k, 2 v, 3 o}) inside the pack buffers
FMD_DEV bf16r* plane(bf16r* q, bf16r* k, bf16r* v, int which) { return which == 0 || which == 3 ? q : (which == 1 ? k : v); }

// Walk over the consecutive d of one (which, head, row) run in the reference buffer: the raw split steps the
// token t and wraps into the next channel c (one division per run); the view split is contiguous in d.
struct RunWalk {
  unsigned t, c, T, ld, off;
  int raw;
  FMD_DEV RunWalk(const Geo& g, int which, int h, int r, int d0) {
    raw = g.raw;
    T = g.rows(which);
    ld = g.parts(which) * g.inner;
    if (raw) {
      const unsigned f = ((unsigned)h * T + r) * g.parts(which) * g.dh + g.slot(which) * g.dh + d0;
      c = f / T;
      t = f - c * T;
      off = 0;
    } else {
      t = c = 0;
      off = (unsigned)r * ld + g.slot(which) * g.inner + h * g.dh + d0;
    }
  }
  FMD_DEV unsigned cur() const { return raw ? t * ld + c : off; }
  FMD_DEV void next() {
    if (raw) {
      if (++t == T) { t = 0; ++c; }
    } else {
      ++off;
    }
  }
};

// src (reference layout) -> canonical [B*heads][rows][DHP] (zero padded), one 8-element run per thread;
// vec: view split with dh % 8 == 0 (one 16-byte load per run)
__global__ void attn_pack_kernel(const bf16r* __restrict__ srcq, const bf16r* __restrict__ srckv, Geo g, int B,
                                 int DHP, int which0, int which1, int vec, bf16r* __restrict__ cq,
                                 bf16r* __restrict__ ck, bf16r* __restrict__ cv) {
  const int runs = DHP / 8;
  for (int w = which0; w <= which1; ++w) {
    const int rows = g.rows(w);
    const long long total = (long long)B * g.heads * rows * runs;
    const bf16r* src = (w == 0 || w == 3 || !g.cross) ? srcq : srckv;
    bf16r* dst = plane(cq, ck, cv, w);
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
      const int run = (int)(i % runs);
      const long long rr = i / runs;
      const int r = (int)(rr % rows);
      const long long bh = rr / rows;
      const int h = (int)(bh % g.heads), b = (int)(bh / g.heads);
      const bf16r* base = src + (size_t)b * g.stride(w);
      const int d0 = run * 8;
      u32x4 v = u32x4{0u, 0u, 0u, 0u};
      if (d0 < g.dh) {
        RunWalk wk(g, w, h, r, d0);
        if (vec) {
          v = *(const u32x4*)(base + wk.cur());
        } else {
          unsigned e16[8];
#pragma unroll
          for (int e = 0; e < 8; ++e) {
            e16[e] = d0 + e < g.dh ? base[wk.cur()] : 0u;
            wk.next();
          }
#pragma unroll
          for (int e = 0; e < 4; ++e) v[e] = e16[2 * e] | (e16[2 * e + 1] << 16);
        }
      }
      *(u32x4*)(dst + (size_t)rr * DHP + d0) = v;
    }
  }
}

// canonical -> reference layout (the d < dh part of each row), one 8-element run per thread
__global__ void attn_unpack_kernel(const bf16r* __restrict__ cq, const bf16r* __restrict__ ck,
                                   const bf16r* __restrict__ cv, Geo g, int B, int DHP, int which0, int which1,
                                   int vec, bf16r* __restrict__ dstq, bf16r* __restrict__ dstkv) {
  const int runs = (g.dh + 7) / 8;
  for (int w = which0; w <= which1; ++w) {
    const int rows = g.rows(w);
    const long long total = (long long)B * g.heads * rows * runs;
    const bf16r* src = w == 0 || w == 3 ? cq : (w == 1 ? ck : cv);
    bf16r* dst = (w == 0 || w == 3 || !g.cross) ? dstq : dstkv;   // self: q, k, v share one [T][3*inner] buffer
    for (long long i = (long long)blockIdx.x * blockDim.x + threadIdx.x; i < total;
         i += (long long)gridDim.x * blockDim.x) {
      const int run = (int)(i % runs);
      const long long rr = i / runs;
      const int r = (int)(rr % rows);
      const long long bh = rr / rows;
      const int h = (int)(bh % g.heads), b = (int)(bh / g.heads);
      bf16r* base = dst + (size_t)b * g.stride(w);
      const int d0 = run * 8;
      const u32x4 v = *(const u32x4*)(src + (size_t)rr * DHP + d0);
      RunWalk wk(g, w, h, r, d0);
      if (vec) {
        *(u32x4*)(base + wk.cur()) = v;
      } else {
#pragma unroll
        for (int e = 0; e < 8; ++e) {
          if (d0 + e < g.dh) base[wk.cur()] = (bf16r)(e & 1 ? v[e >> 1] >> 16 : v[e >> 1] & 0xffffu);
          wk.next();
        }
      }
    }
  }
}

// Raw head split as a tile transpose.  The raw reshape reads the [T][P*inner] buffer as its transpose
// [P*inner][T] flattened: element (c, t) sits at flat f = c*T + t = ((h*T + r)*P + slot)*dh + d, i.e. the
// canonical order up to the plane split.  A workgroup moves a 64-token x 64-channel tile through LDS: 16-byte
// coalesced rows on the reference side, 16-byte runs of one canonical row (dh | 64, T % 64 == 0) on the other.
constexpr int RT = 64, RTLD = RT + 8;

struct RawSet {
  const bf16r* src;   // pack: reference buffer; unpack: unused
  bf16r* dst;         // unpack: reference buffer; pack: unused
  bf16r* pl[3];       // canonical planes of slots 0..P-1
  int P, T, heads, dh, DHP;
  size_t stride;      // elements per batch in the reference buffer
};

FMD_DEV bf16r* raw_canon(const RawSet& st, int b, unsigned f) {
  const unsigned d0 = f % st.dh, rest = f / st.dh;
  const unsigned slot = rest % st.P, hr = rest / st.P;
  const unsigned h = hr / st.T, r = hr - h * st.T;
  return st.pl[slot] + (((size_t)b * st.heads + h) * st.T + r) * st.DHP + d0;
}

__global__ __launch_bounds__(256) void attn_pack_raw_tile(RawSet st) {
  __shared__ __attribute__((aligned(16))) bf16r tile[RT * RTLD];   // [channel][token]
  const int t0 = blockIdx.x * RT, c0 = blockIdx.y * RT, b = blockIdx.z;
  const int ld = st.P * st.heads * st.dh;
  const bf16r* src = st.src + (size_t)b * st.stride;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = threadIdx.x + 256 * j, t = k >> 3, cc = (k & 7) * 8;
    const u32x4 v = *(const u32x4*)(src + (size_t)(t0 + t) * ld + c0 + cc);
#pragma unroll
    for (int e = 0; e < 8; ++e) tile[(cc + e) * RTLD + t] = (bf16r)(e & 1 ? v[e >> 1] >> 16 : v[e >> 1] & 0xffffu);
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = threadIdx.x + 256 * j, c = k >> 3, tc = (k & 7) * 8;
    const unsigned f = (unsigned)(c0 + c) * st.T + t0 + tc;
    *(u32x4*)raw_canon(st, b, f) = *(const u32x4*)(tile + c * RTLD + tc);
  }
}

__global__ __launch_bounds__(256) void attn_unpack_raw_tile(RawSet st) {
  __shared__ __attribute__((aligned(16))) bf16r tile[RT * RTLD];   // [channel][token]
  const int t0 = blockIdx.x * RT, c0 = blockIdx.y * RT, b = blockIdx.z;
  const int ld = st.P * st.heads * st.dh;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = threadIdx.x + 256 * j, c = k >> 3, tc = (k & 7) * 8;
    const unsigned f = (unsigned)(c0 + c) * st.T + t0 + tc;
    *(u32x4*)(tile + c * RTLD + tc) = *(const u32x4*)raw_canon(st, b, f);
  }
  __syncthreads();
  bf16r* dst = st.dst + (size_t)b * st.stride;
#pragma unroll
  for (int j = 0; j < 2; ++j) {
    const int k = threadIdx.x + 256 * j, t = k >> 3, cc = (k & 7) * 8;
    u32x4 v;
#pragma unroll
    for (int e = 0; e < 4; ++e)
      v[e] = (unsigned)tile[(cc + 2 * e) * RTLD + t] | ((unsigned)tile[(cc + 2 * e + 1) * RTLD + t] << 16);
    *(u32x4*)(dst + (size_t)(t0 + t) * ld + c0 + cc) = v;
  }
}

// ------------------------------------------------------------------ MFMA kernels (canonical layout)
template <int DHP>
struct Blk {
  static constexpr int LD = DHP + 8;           // LDS row pitch (elements): 16-byte-slot-distinct rows
  static constexpr int NS = DHP / 16;          // 16-deep k-steps over the head dim
  static constexpr int NB = DHP > 32 ? DHP / 32 : 1;   // 32-row blocks of a transposed (d-major) accumulator
};

// 32 rows x DHP block of a canonical plane into LDS rows [32][LD] (rows past `valid` zero); 256 threads
template <int DHP>
FMD_DEV void stage_rows(bf16r* lds, const bf16r* __restrict__ src, int row0, int valid) {
  constexpr int RUNS = DHP / 8;
  for (int i = threadIdx.x; i < 32 * RUNS; i += 256) {
    const int r = i / RUNS, run = i - (i / RUNS) * RUNS;
    u32x4 v = u32x4{0u, 0u, 0u, 0u};
    if (r < valid) v = *(const u32x4*)(src + (size_t)(row0 + r) * DHP + run * 8);
    *(u32x4*)(lds + r * Blk<DHP>::LD + run * 8) = v;
  }
}

// A fragment of rows = the 32 staged rows, k = head dim (k-step s): lane (r, h) reads row r, d = 16s + 8h
template <int DHP>
FMD_DEV bf16x8 frag_rows(const bf16r* lds, int s) {
  const int lane = threadIdx.x & 63;
  return *(const bf16x8*)(lds + (lane & 31) * Blk<DHP>::LD + 16 * s + 8 * (lane >> 5));
}

// A fragment of the transposed block (rows = head dim d in [32 db, 32 db + 32), k = the 32 staged rows) for
// the accumulator-operand k order of k-step s: element j <-> staged row 16s + 8(j>>2) + 4h + (j&3)
template <int DHP>
FMD_DEV bf16x8 frag_tr(const bf16r* lds, int db, int s) {
  const int lane = threadIdx.x & 63;
  const int G = lane >> 4, i = lane & 15, qq = i >> 2, p = i & 3;
  const int h = G >> 1;
  const int col = 32 * db + 16 * (G & 1) + 4 * p;
  const int r0 = 16 * s + 4 * h + qq;
  // every lane reads (the gather needs EXEC all ones); DHP = 16: the second half of the d rows is padding, read
  // in bounds from columns 0..15 and zeroed
  const bool pad = 32 * db + 16 * (G & 1) >= DHP;
  const int c = pad ? 4 * p : col;
  s16x4 lo = ds_read_tr16(lds + r0 * Blk<DHP>::LD + c);
  s16x4 hi = ds_read_tr16(lds + (r0 + 8) * Blk<DHP>::LD + c);
  if (pad) { lo = s16x4{0, 0, 0, 0}; hi = s16x4{0, 0, 0, 0}; }
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

// fragment of one canonical row (this lane's column r) for k-step s, from global memory (zero if row invalid)
template <int DHP>
FMD_DEV bf16x8 frag_row_global(const bf16r* __restrict__ plane_bh, int row, bool ok, int s) {
  const int h = (threadIdx.x & 63) >> 5;
  if (!ok) {
    bf16x8 z;
#pragma unroll
    for (int j = 0; j < 8; ++j) z[j] = (__bf16)0.f;
    return z;
  }
  return *(const bf16x8*)(plane_bh + (size_t)row * DHP + 16 * s + 8 * h);
}

// accumulator registers 8s..8s+7 -> bf16 operand fragment of k-step s
FMD_DEV bf16x8 acc_frag(const f32x16& a, int s) {
  bf16x8 f;
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = (__bf16)a[8 * s + j];
  return f;
}

FMD_DEV int acc_row(int i) { return (i & 3) + 8 * (i >> 2) + 4 * ((threadIdx.x & 63) >> 5); }

// write a transposed accumulator block (rows d = 32 db + acc_row(i), column = this lane's row) to a canonical row
template <int DHP>
FMD_DEV void store_tr(bf16r* __restrict__ dst_row, const f32x16& a, int db, float mul) {
#pragma unroll
  for (int g4 = 0; g4 < 4; ++g4) {
    const int d = 32 * db + 8 * g4 + 4 * ((threadIdx.x & 63) >> 5);
    if (d < DHP) {
      u32x2 o;
      o[0] = pack2(a[4 * g4] * mul, a[4 * g4 + 1] * mul);
      o[1] = pack2(a[4 * g4 + 2] * mul, a[4 * g4 + 3] * mul);
      *(u32x2*)(dst_row + d) = o;
    }
  }
}

// Staging of R = 32*KS rows x DHP of a canonical plane through registers (prefetch of the next block while the
// current one is in use): each of the NT = 256*KS threads owns at most one 16-byte run.
template <int DHP, int NT, int R>
struct Stager {
  static constexpr int RUNS = DHP / 8;
  static_assert(R * RUNS <= NT, "one run per thread");
  u32x4 v;
  bool own;
  int r, run;
  FMD_DEV Stager() : own(threadIdx.x < R * RUNS), r(threadIdx.x / RUNS), run(threadIdx.x % RUNS) {}
  FMD_DEV void load(const bf16r* __restrict__ src, int row0, int valid) {
    v = u32x4{0u, 0u, 0u, 0u};
    if (own && r < valid) v = *(const u32x4*)(src + (size_t)(row0 + r) * DHP + run * 8);
  }
  FMD_DEV void store(bf16r* lds) const {
    if (own) *(u32x4*)(lds + r * Blk<DHP>::LD + run * 8) = v;
  }
};

template <int DHP, int KS, int PARTF>
struct Smem {
  static constexpr int TILE = 32 * KS * Blk<DHP>::LD;                  // elements of one staged tensor block
  static constexpr int STAGE = 2 * 2 * TILE * 2;                       // bytes: 2 buffers x 2 tensors
  static constexpr int COMB = KS > 1 ? (KS / 2) * 4 * PARTF * 64 * 4 : 0;   // bytes of the split-combine slots
  static constexpr int BYTES = STAGE > COMB ? STAGE : COMB;
};

// Forward: grid (ceil(Tq / 128), B*heads), 256*KS threads.  Wave w: query block w & 3 (32 queries), key split
// w >> 2 (keys 32*split .. +31 of every staged block of 32*KS keys); the KS partial (m, l, O^T) are merged in LDS.
template <int DHP, int KS>
__global__ __launch_bounds__(256 * KS) void attn_mfma_fwd(const bf16r* __restrict__ cq, const bf16r* __restrict__ ck,
                                                          const bf16r* __restrict__ cv, int Tq, int Tk, float scale,
                                                          bf16r* __restrict__ co, float* __restrict__ lse) {
  using BK = Blk<DHP>;
  constexpr int PARTF = BK::NB * 16 + 2;
  using SM = Smem<DHP, KS, PARTF>;
  constexpr int KB = 32 * KS, TILE = SM::TILE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM::BYTES];
  bf16r* sb = (bf16r*)smem;
  const int bh = blockIdx.y, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qw = wid & 3, ks = wid >> 2, col = lane & 31;
  const int q = blockIdx.x * 128 + qw * 32 + col;
  const bool qok = q < Tq;
  const bf16r* qb = cq + (size_t)bh * Tq * DHP;
  const bf16r* kb = ck + (size_t)bh * Tk * DHP;
  const bf16r* vb = cv + (size_t)bh * Tk * DHP;
  bf16x8 qf[BK::NS];
#pragma unroll
  for (int s = 0; s < BK::NS; ++s) qf[s] = frag_row_global<DHP>(qb, q, qok, s);
  const float sl2 = scale * LOG2E;
  f32x16 ob[BK::NB];
#pragma unroll
  for (int db = 0; db < BK::NB; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) ob[db][i] = 0.f;
  float m = -INFINITY, l = 0.f;
  Stager<DHP, 256 * KS, KB> sk, sv;
  const int nblk = (Tk + KB - 1) / KB;
  sk.load(kb, 0, Tk);
  sv.load(vb, 0, Tk);
  sk.store(sb);
  sv.store(sb + TILE);
  __syncthreads();
  for (int it = 0; it < nblk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nblk) {
      sk.load(kb, (it + 1) * KB, Tk - (it + 1) * KB);
      sv.load(vb, (it + 1) * KB, Tk - (it + 1) * KB);
    }
    const int kv = min(32, Tk - (it * KB + ks * 32));
    if (kv > 0) {   // wave-uniform
      const bf16r* kl = sb + (2 * cur) * TILE + ks * 32 * BK::LD;
      const bf16r* vl = sb + (2 * cur + 1) * TILE + ks * 32 * BK::LD;
      f32x16 st;
#pragma unroll
      for (int i = 0; i < 16; ++i) st[i] = 0.f;
#pragma unroll
      for (int s = 0; s < BK::NS; ++s) st = mfma32(frag_rows<DHP>(kl, s), qf[s], st);
      float bm = -INFINITY;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] = acc_row(i) < kv ? st[i] * sl2 : -INFINITY;
        bm = fmaxf(bm, st[i]);
      }
      bm = fmaxf(bm, __shfl_xor(bm, 32, 64));
      const float mn = fmaxf(m, bm);
      const float corr = exp2f(m - mn);
      float ps = 0.f;
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        st[i] = exp2f(st[i] - mn);
        ps += st[i];
      }
      ps += __shfl_xor(ps, 32, 64);
      l = l * corr + ps;
      m = mn;
#pragma unroll
      for (int db = 0; db < BK::NB; ++db)
#pragma unroll
        for (int i = 0; i < 16; ++i) ob[db][i] *= corr;
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(st, s);
#pragma unroll
        for (int db = 0; db < BK::NB; ++db) ob[db] = mfma32(frag_tr<DHP>(vl, db, s), pf, ob[db]);
      }
    }
    if (it + 1 < nblk) {
      sk.store(sb + 2 * (cur ^ 1) * TILE);
      sv.store(sb + (2 * (cur ^ 1) + 1) * TILE);
    }
    __syncthreads();
  }
  if constexpr (KS > 1) {
    float* part = (float*)smem;
#pragma unroll
    for (int step = KS / 2; step >= 1; step >>= 1) {
      if (ks >= step && ks < 2 * step) {
        float* p = part + ((ks - step) * 4 + qw) * PARTF * 64 + lane;
#pragma unroll
        for (int db = 0; db < BK::NB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) p[(db * 16 + i) * 64] = ob[db][i];
        p[(PARTF - 2) * 64] = m;
        p[(PARTF - 1) * 64] = l;
      }
      __syncthreads();
      if (ks < step) {
        const float* p = part + (ks * 4 + qw) * PARTF * 64 + lane;
        const float mo = p[(PARTF - 2) * 64], lo = p[(PARTF - 1) * 64];
        const float mn = fmaxf(m, mo);
        const float fa = m == -INFINITY ? 0.f : exp2f(m - mn);
        const float fb = mo == -INFINITY ? 0.f : exp2f(mo - mn);
#pragma unroll
        for (int db = 0; db < BK::NB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) ob[db][i] = ob[db][i] * fa + p[(db * 16 + i) * 64] * fb;
        l = l * fa + lo * fb;
        m = mn;
      }
      __syncthreads();
    }
  }
  if (ks != 0 || !qok) return;
  const float inv = 1.f / l;
#pragma unroll
  for (int db = 0; db < BK::NB; ++db) store_tr<DHP>(co + ((size_t)bh * Tq + q) * DHP, ob[db], db, inv);
  if ((lane >> 5) == 0) lse[(size_t)bh * Tq + q] = (m + log2f(l)) * LN2;
}

// dQ: grid (ceil(Tq / 128), B*heads), 256*KS threads, waves as in the forward (partial dQ^T summed in LDS);
// also writes delta = rowsum(dO * O)
template <int DHP, int KS>
__global__ __launch_bounds__(256 * KS) void attn_mfma_bwd_q(const bf16r* __restrict__ cq, const bf16r* __restrict__ ck,
                                                            const bf16r* __restrict__ cv, const bf16r* __restrict__ co,
                                                            const bf16r* __restrict__ cdo, const float* __restrict__ lse,
                                                            int Tq, int Tk, float scale, float* __restrict__ delta,
                                                            bf16r* __restrict__ cdq) {
  using BK = Blk<DHP>;
  constexpr int PARTF = BK::NB * 16;
  using SM = Smem<DHP, KS, PARTF>;
  constexpr int KB = 32 * KS, TILE = SM::TILE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM::BYTES];
  bf16r* sb = (bf16r*)smem;
  const int bh = blockIdx.y, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int qw = wid & 3, ks = wid >> 2, col = lane & 31;
  const int q = blockIdx.x * 128 + qw * 32 + col;
  const bool qok = q < Tq;
  const size_t qoff = (size_t)bh * Tq * DHP;
  const bf16r* kb = ck + (size_t)bh * Tk * DHP;
  const bf16r* vb = cv + (size_t)bh * Tk * DHP;
  bf16x8 qf[BK::NS], dof[BK::NS];
  float dl = 0.f;
#pragma unroll
  for (int s = 0; s < BK::NS; ++s) {
    qf[s] = frag_row_global<DHP>(cq + qoff, q, qok, s);
    dof[s] = frag_row_global<DHP>(cdo + qoff, q, qok, s);
    const bf16x8 of = frag_row_global<DHP>(co + qoff, q, qok, s);
#pragma unroll
    for (int j = 0; j < 8; ++j) dl += (float)dof[s][j] * (float)of[j];
  }
  dl += __shfl_xor(dl, 32, 64);
  const float L2 = qok ? lse[(size_t)bh * Tq + q] * LOG2E : 0.f;
  const float sl2 = scale * LOG2E;
  f32x16 dq[BK::NB];
#pragma unroll
  for (int db = 0; db < BK::NB; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) dq[db][i] = 0.f;
  Stager<DHP, 256 * KS, KB> sk, sv;
  const int nblk = (Tk + KB - 1) / KB;
  sk.load(kb, 0, Tk);
  sv.load(vb, 0, Tk);
  sk.store(sb);
  sv.store(sb + TILE);
  __syncthreads();
  for (int it = 0; it < nblk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nblk) {
      sk.load(kb, (it + 1) * KB, Tk - (it + 1) * KB);
      sv.load(vb, (it + 1) * KB, Tk - (it + 1) * KB);
    }
    const int kv = min(32, Tk - (it * KB + ks * 32));
    if (kv > 0) {
      const bf16r* kl = sb + (2 * cur) * TILE + ks * 32 * BK::LD;
      const bf16r* vl = sb + (2 * cur + 1) * TILE + ks * 32 * BK::LD;
      f32x16 st, dp;
#pragma unroll
      for (int i = 0; i < 16; ++i) { st[i] = 0.f; dp[i] = 0.f; }
#pragma unroll
      for (int s = 0; s < BK::NS; ++s) {
        st = mfma32(frag_rows<DHP>(kl, s), qf[s], st);
        dp = mfma32(frag_rows<DHP>(vl, s), dof[s], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const float p = (acc_row(i) < kv && qok) ? exp2f(st[i] * sl2 - L2) : 0.f;
        st[i] = p * (dp[i] - dl);   // dS^T
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 df = acc_frag(st, s);
#pragma unroll
        for (int db = 0; db < BK::NB; ++db) dq[db] = mfma32(frag_tr<DHP>(kl, db, s), df, dq[db]);
      }
    }
    if (it + 1 < nblk) {
      sk.store(sb + 2 * (cur ^ 1) * TILE);
      sv.store(sb + (2 * (cur ^ 1) + 1) * TILE);
    }
    __syncthreads();
  }
  if constexpr (KS > 1) {
    float* part = (float*)smem;
#pragma unroll
    for (int step = KS / 2; step >= 1; step >>= 1) {
      if (ks >= step && ks < 2 * step) {
        float* p = part + ((ks - step) * 4 + qw) * PARTF * 64 + lane;
#pragma unroll
        for (int db = 0; db < BK::NB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) p[(db * 16 + i) * 64] = dq[db][i];
      }
      __syncthreads();
      if (ks < step) {
        const float* p = part + (ks * 4 + qw) * PARTF * 64 + lane;
#pragma unroll
        for (int db = 0; db < BK::NB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) dq[db][i] += p[(db * 16 + i) * 64];
      }
      __syncthreads();
    }
  }
  if (ks != 0 || !qok) return;
#pragma unroll
  for (int db = 0; db < BK::NB; ++db) store_tr<DHP>(cdq + qoff + (size_t)q * DHP, dq[db], db, scale);
  if ((lane >> 5) == 0) delta[(size_t)bh * Tq + q] = dl;
}

// dK, dV: grid (ceil(Tk / 128), B*heads), 256*KS threads.  Wave w: key block w & 3 (32 keys), query split w >> 2 of
// every staged block of 32*KS queries; partial dK^T, dV^T summed in LDS.
template <int DHP, int KS>
__global__ __launch_bounds__(256 * KS) void attn_mfma_bwd_kv(const bf16r* __restrict__ cq, const bf16r* __restrict__ ck,
                                                             const bf16r* __restrict__ cv, const bf16r* __restrict__ cdo,
                                                             const float* __restrict__ lse,
                                                             const float* __restrict__ delta, int Tq, int Tk,
                                                             float scale, bf16r* __restrict__ cdk,
                                                             bf16r* __restrict__ cdv) {
  using BK = Blk<DHP>;
  constexpr int PARTF = 2 * BK::NB * 16;
  using SM = Smem<DHP, KS, PARTF>;
  static_assert(SM::BYTES <= 65536, "split-combine slots exceed 64 KB");
  constexpr int QB = 32 * KS, TILE = SM::TILE;
  __shared__ __attribute__((aligned(16))) unsigned char smem[SM::BYTES];
  __shared__ float lsl[2][QB], dll[2][QB];
  bf16r* sb = (bf16r*)smem;
  const int bh = blockIdx.y, wid = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int kw = wid & 3, ks = wid >> 2, col = lane & 31;
  const int key = blockIdx.x * 128 + kw * 32 + col;
  const bool kok = key < Tk;
  const size_t koff = (size_t)bh * Tk * DHP;
  const bf16r* qb = cq + (size_t)bh * Tq * DHP;
  const bf16r* dob = cdo + (size_t)bh * Tq * DHP;
  const float* lb = lse + (size_t)bh * Tq;
  const float* dlb = delta + (size_t)bh * Tq;
  bf16x8 kf[BK::NS], vf[BK::NS];
#pragma unroll
  for (int s = 0; s < BK::NS; ++s) {
    kf[s] = frag_row_global<DHP>(ck + koff, key, kok, s);
    vf[s] = frag_row_global<DHP>(cv + koff, key, kok, s);
  }
  const float sl2 = scale * LOG2E;
  f32x16 dk[BK::NB], dv[BK::NB];
#pragma unroll
  for (int db = 0; db < BK::NB; ++db)
#pragma unroll
    for (int i = 0; i < 16; ++i) { dk[db][i] = 0.f; dv[db][i] = 0.f; }
  Stager<DHP, 256 * KS, QB> sq, sd;
  const bool ownrow = threadIdx.x < QB;
  float rl = 0.f, rd = 0.f;
  auto load_rows = [&](int q0) {
    const int n = Tq - q0;
    rl = ownrow && (int)threadIdx.x < n ? lb[q0 + threadIdx.x] * LOG2E : INFINITY;
    rd = ownrow && (int)threadIdx.x < n ? dlb[q0 + threadIdx.x] : 0.f;
  };
  const int nblk = (Tq + QB - 1) / QB;
  sq.load(qb, 0, Tq);
  sd.load(dob, 0, Tq);
  load_rows(0);
  sq.store(sb);
  sd.store(sb + TILE);
  if (ownrow) { lsl[0][threadIdx.x] = rl; dll[0][threadIdx.x] = rd; }
  __syncthreads();
  for (int it = 0; it < nblk; ++it) {
    const int cur = it & 1;
    if (it + 1 < nblk) {
      sq.load(qb, (it + 1) * QB, Tq - (it + 1) * QB);
      sd.load(dob, (it + 1) * QB, Tq - (it + 1) * QB);
      load_rows((it + 1) * QB);
    }
    const int qv = min(32, Tq - (it * QB + ks * 32));
    if (qv > 0) {
      const bf16r* ql = sb + (2 * cur) * TILE + ks * 32 * BK::LD;
      const bf16r* dol = sb + (2 * cur + 1) * TILE + ks * 32 * BK::LD;
      const float* ls = lsl[cur] + ks * 32;
      const float* ds = dll[cur] + ks * 32;
      f32x16 st, dp;   // rows = queries, columns = keys
#pragma unroll
      for (int i = 0; i < 16; ++i) { st[i] = 0.f; dp[i] = 0.f; }
#pragma unroll
      for (int s = 0; s < BK::NS; ++s) {
        st = mfma32(frag_rows<DHP>(ql, s), kf[s], st);
        dp = mfma32(frag_rows<DHP>(dol, s), vf[s], dp);
      }
#pragma unroll
      for (int i = 0; i < 16; ++i) {
        const int r = acc_row(i);
        const float p = kok ? exp2f(st[i] * sl2 - ls[r]) : 0.f;   // rows past Tq: lse = +inf -> p = 0
        dp[i] = p * (dp[i] - ds[r]);   // dS
        st[i] = p;                     // P
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pf = acc_frag(st, s), df = acc_frag(dp, s);
#pragma unroll
        for (int db = 0; db < BK::NB; ++db) {
          dv[db] = mfma32(frag_tr<DHP>(dol, db, s), pf, dv[db]);
          dk[db] = mfma32(frag_tr<DHP>(ql, db, s), df, dk[db]);
        }
      }
    }
    if (it + 1 < nblk) {
      sq.store(sb + 2 * (cur ^ 1) * TILE);
      sd.store(sb + (2 * (cur ^ 1) + 1) * TILE);
      if (ownrow) { lsl[cur ^ 1][threadIdx.x] = rl; dll[cur ^ 1][threadIdx.x] = rd; }
    }
    __syncthreads();
  }
  if constexpr (KS > 1) {
    float* part = (float*)smem;
#pragma unroll
    for (int step = KS / 2; step >= 1; step >>= 1) {
      if (ks >= step && ks < 2 * step) {
        float* p = part + ((ks - step) * 4 + kw) * PARTF * 64 + lane;
#pragma unroll
        for (int db = 0; db < BK::NB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            p[(db * 16 + i) * 64] = dk[db][i];
            p[((BK::NB + db) * 16 + i) * 64] = dv[db][i];
          }
      }
      __syncthreads();
      if (ks < step) {
        const float* p = part + (ks * 4 + kw) * PARTF * 64 + lane;
#pragma unroll
        for (int db = 0; db < BK::NB; ++db)
#pragma unroll
          for (int i = 0; i < 16; ++i) {
            dk[db][i] += p[(db * 16 + i) * 64];
            dv[db][i] += p[((BK::NB + db) * 16 + i) * 64];
          }
      }
      __syncthreads();
    }
  }
  if (ks != 0 || !kok) return;
#pragma unroll
  for (int db = 0; db < BK::NB; ++db) {
    store_tr<DHP>(cdk + koff + (size_t)key * DHP, dk[db], db, scale);
    store_tr<DHP>(cdv + koff + (size_t)key * DHP, dv[db], db, 1.f);
  }
}

int dhp_of(int dh) { return dh <= 16 ? 16 : (dh <= 32 ? 32 : 64); }

template <typename F>
int dispatch_dhp(int dhp, F&& f) {
  if (dhp == 16) return f(std::integral_constant<int, 16>{});
  if (dhp == 32) return f(std::integral_constant<int, 32>{});
  return f(std::integral_constant<int, 64>{});
}

int grid_for(long long work) {
  long long b = (work + 255) / 256;
  return (int)(b < 1 ? 1 : (b > 16384 ? 16384 : b));
}

// Launch the raw tile transpose for planes which0..which1 if the shape allows it (raw split, dh in {16, 32, 64},
// tokens % 64 == 0, channels % 64 == 0, whole slot sets); returns false to fall back to the run kernels.
bool raw_sets(const Geo& g, int B, int which0, int which1, const void* src_q, const void* src_kv, void* dst_q,
              void* dst_kv, bf16r* cq, bf16r* ck, bf16r* cv, bool pack, hipStream_t s) {
  if (!g.raw || !(g.dh == 16 || g.dh == 32 || g.dh == 64) || B > 65535) return false;
  struct Set { int which0, which1, P, T; const void* src; void* dst; bf16r* pl[3]; };
  Set sets[2];
  int n = 0;
  if (which0 == 3 && which1 == 3) {
    sets[n++] = Set{3, 3, 1, g.Tq, src_q, dst_q, {cq, nullptr, nullptr}};
  } else if (which1 <= 2 && !g.cross && which0 == 0 && which1 == 2) {
    sets[n++] = Set{0, 2, 3, g.Tq, src_q, dst_q, {cq, ck, cv}};
  } else if (which1 <= 2 && g.cross) {
    if (which0 == 0) sets[n++] = Set{0, 0, 1, g.Tq, src_q, dst_q, {cq, nullptr, nullptr}};
    if (which1 == 2 && which0 <= 1) sets[n++] = Set{1, 2, 2, g.Tk, src_kv, dst_kv, {ck, cv, nullptr}};
    if (which1 == 1) return false;
  } else {
    return false;
  }
  for (int i = 0; i < n; ++i)
    if (sets[i].T % RT || (sets[i].P * g.inner) % RT) return false;
  for (int i = 0; i < n; ++i) {
    RawSet st;
    st.src = (const bf16r*)sets[i].src;
    st.dst = (bf16r*)sets[i].dst;
    for (int k = 0; k < 3; ++k) st.pl[k] = sets[i].pl[k];
    st.P = sets[i].P;
    st.T = sets[i].T;
    st.heads = g.heads;
    st.dh = g.dh;
    st.DHP = dhp_of(g.dh);
    st.stride = (size_t)sets[i].T * sets[i].P * g.inner;
    const dim3 grid(sets[i].T / RT, sets[i].P * g.inner / RT, B);
    if (pack)
      hipLaunchKernelGGL(attn_pack_raw_tile, grid, dim3(256), 0, s, st);
    else
      hipLaunchKernelGGL(attn_unpack_raw_tile, grid, dim3(256), 0, s, st);
  }
  return true;
}

bool geo_ok(const Geo& g, int B) {
  return B > 0 && g.Tq > 0 && g.Tk > 0 && g.heads > 0 && g.dh > 0 && g.dh <= 64 &&
         g.stride(0) < (1ull << 32) && g.stride(1) < (1ull << 32) && (size_t)g.Tq * g.inner < (1ull << 32);
}

}  // namespace

extern "C" int32_t fmd_attn_head_pad(int32_t dh) { return dh < 1 || dh > 64 ? -1 : dhp_of(dh); }

extern "C" int fmd_attn_pack(const void* src_q, const void* src_kv, int32_t B, int32_t Tq, int32_t Tk, int32_t heads,
                             int32_t dh, int32_t raw, int32_t cross, int32_t which0, int32_t which1, void* cq,
                             void* ck, void* cv, fmd_stream_t s) {
  const Geo g{Tq, Tk, heads, dh, heads * dh, raw, cross};
  if (!geo_ok(g, B) || which0 < 0 || which1 > 3 || which0 > which1) return -1;
  if (raw_sets(g, B, which0, which1, src_q, src_kv, nullptr, nullptr, (bf16r*)cq, (bf16r*)ck, (bf16r*)cv, true,
               (hipStream_t)s))
    return (int)hipGetLastError();
  const long long work = (long long)B * heads * (Tq + 2LL * Tk) * (dhp_of(dh) / 8);
  hipLaunchKernelGGL(attn_pack_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)s, (const bf16r*)src_q,
                     (const bf16r*)src_kv, g, B, dhp_of(dh), which0, which1, (int)(!raw && dh % 8 == 0), (bf16r*)cq,
                     (bf16r*)ck, (bf16r*)cv);
  return (int)hipGetLastError();
}

extern "C" int fmd_attn_unpack(const void* cq, const void* ck, const void* cv, int32_t B, int32_t Tq, int32_t Tk,
                               int32_t heads, int32_t dh, int32_t raw, int32_t cross, int32_t which0, int32_t which1,
                               void* dst_q, void* dst_kv, fmd_stream_t s) {
  const Geo g{Tq, Tk, heads, dh, heads * dh, raw, cross};
  if (!geo_ok(g, B) || which0 < 0 || which1 > 3 || which0 > which1) return -1;
  if (raw_sets(g, B, which0, which1, nullptr, nullptr, dst_q, dst_kv, (bf16r*)cq, (bf16r*)ck, (bf16r*)cv, false,
               (hipStream_t)s))
    return (int)hipGetLastError();
  const long long work = (long long)B * heads * (Tq + 2LL * Tk) * ((dh + 7) / 8);
  hipLaunchKernelGGL(attn_unpack_kernel, dim3(grid_for(work)), dim3(256), 0, (hipStream_t)s, (const bf16r*)cq,
                     (const bf16r*)ck, (const bf16r*)cv, g, B, dhp_of(dh), which0, which1, (int)(!raw && dh % 8 == 0),
                     (bf16r*)dst_q, (bf16r*)dst_kv);
  return (int)hipGetLastError();
}

namespace {

// key splits of the forward / dQ kernels: enough waves for small grids, one split for short key ranges
int ks_q(int Tq, int Tk, int BH) {
  const long long nwg = (long long)((Tq + 127) / 128) * BH;
  if (Tk > 128 && nwg < 512) return 4;
  return Tk > 32 ? 2 : 1;
}

template <typename F>
int dispatch_ks(int ks, F&& f) {
  if (ks == 4) return f(std::integral_constant<int, 4>{});
  if (ks == 2) return f(std::integral_constant<int, 2>{});
  return f(std::integral_constant<int, 1>{});
}

}  // namespace

extern "C" int fmd_attn_mfma_fwd(const void* cq, const void* ck, const void* cv, int32_t BH, int32_t Tq, int32_t Tk,
                                 int32_t dh, void* co, float* lse, fmd_stream_t s) {
  if (BH < 1 || Tq < 1 || Tk < 1 || dh < 1 || dh > 64) return -1;
  const float scale = 1.0f / sqrtf((float)dh);
  return dispatch_dhp(dhp_of(dh), [&](auto dhp) {
    constexpr int D = decltype(dhp)::value;
    return dispatch_ks(ks_q(Tq, Tk, BH), [&](auto ksc) {
      constexpr int KS = decltype(ksc)::value;
      hipLaunchKernelGGL((attn_mfma_fwd<D, KS>), dim3((Tq + 127) / 128, BH), dim3(256 * KS), 0, (hipStream_t)s,
                         (const bf16r*)cq, (const bf16r*)ck, (const bf16r*)cv, Tq, Tk, scale, (bf16r*)co, lse);
      return (int)hipGetLastError();
    });
  });
}

extern "C" int fmd_attn_mfma_bwd(const void* cq, const void* ck, const void* cv, const void* co, const void* cdo,
                                 const float* lse, float* delta, int32_t BH, int32_t Tq, int32_t Tk, int32_t dh,
                                 void* cdq, void* cdk, void* cdv, fmd_stream_t s) {
  if (BH < 1 || Tq < 1 || Tk < 1 || dh < 1 || dh > 64) return -1;
  const float scale = 1.0f / sqrtf((float)dh);
  return dispatch_dhp(dhp_of(dh), [&](auto dhp) {
    constexpr int D = decltype(dhp)::value;
    // 1024-thread dQ at DHP 64 would cap the wave at 128 VGPRs and spill: at most 2 splits there
    int rc = dispatch_ks(D == 64 ? min(2, ks_q(Tq, Tk, BH)) : ks_q(Tq, Tk, BH), [&](auto ksc) {
      constexpr int KS = decltype(ksc)::value;
      hipLaunchKernelGGL((attn_mfma_bwd_q<D, KS>), dim3((Tq + 127) / 128, BH), dim3(256 * KS), 0, (hipStream_t)s,
                         (const bf16r*)cq, (const bf16r*)ck, (const bf16r*)cv, (const bf16r*)co, (const bf16r*)cdo,
                         lse, Tq, Tk, scale, delta, (bf16r*)cdq);
      return (int)hipGetLastError();
    });
    if (rc) return rc;
    return dispatch_ks(Tq > 32 ? 2 : 1, [&](auto ksc) {
      constexpr int KS = decltype(ksc)::value;
      if constexpr (KS <= 2) {
        hipLaunchKernelGGL((attn_mfma_bwd_kv<D, KS>), dim3((Tk + 127) / 128, BH), dim3(256 * KS), 0,
                           (hipStream_t)s, (const bf16r*)cq, (const bf16r*)ck, (const bf16r*)cv, (const bf16r*)cdo,
                           lse, delta, Tq, Tk, scale, (bf16r*)cdk, (bf16r*)cdv);
        return (int)hipGetLastError();
      }
      return -1;
    });
  });
}
